#!/bin/bash
# Round 3: per-phase clock shares of the matrix kernels (diag variants) and the
# PMC passes of one variant on config B (bench.py --variant V).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python scripts/ab_variants.py --config B --variants ${DVARIANTS:-169,165} --rounds 1 > gpurun_out/ab_diag_B.json 2>&1 || { echo "diag B failed"; exit 1; }
timeout -k 10 200 python scripts/ab_variants.py --config C --width 480 --height 270 --frames 2 --variants ${DVARIANTS:-169,165} --rounds 1 > gpurun_out/ab_diag_C.json 2>&1 || { echo "diag C failed"; exit 1; }
if [ -n "${PMC_VARIANT}" ]; then
  BENCH_ARGS="--variant ${PMC_VARIANT}" EXTRA_MFMA=1 bash scripts/profile_pmc.sh > gpurun_out/pmc.log 2>&1 || { echo "pmc failed"; exit 1; }
fi
echo "all ok"
