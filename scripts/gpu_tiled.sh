#!/bin/bash
# Tiled (LDS) brute variants: parity on config B slabs, A/B on config C (2 spp).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "brute_variants or tiled" > gpurun_out/t.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 400 python scripts/ab_variants.py --config C --rays 2 --frames 1 --variants ${VARIANTS:-86,87,89} --rounds 2 > gpurun_out/ab_C.json 2>&1 || { echo "ab C failed"; exit 1; }
echo "all ok"
