#!/bin/bash
# Round 3: config E (1M triangles, mirror box, 16 bounces) on a reduced image:
# the scalar LDS-tiled kernel vs the k16 matrix kernels (global records / LDS tiles).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python scripts/ab_variants.py --config E --width ${EW:-480} --height ${EH:-270} --variants ${EVARIANTS:-86,200,186} --rounds 1 > gpurun_out/ab_E.json 2>&1 || { echo "ab E failed"; exit 1; }
echo "all ok"
