#!/bin/bash
# Matrix-filter threshold T = 2^-10 / 2^-12 / 2^-14 (Omax + A + 1): parity of
# the tightened variants (experiment build), interleaved A/B on config B and a
# config C sample, and the survivor counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export RT2_LIB=exp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py -x -v --timeout 120 --timeout-method thread -k "${TESTK:-v154 or v155 or v156}" > gpurun_out/tshift_tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 240 python scripts/ab_variants.py --config B --variants ${VARIANTS:-152,154,155} --rounds 3 > gpurun_out/ab_B_t.json 2>&1 || { echo "ab B failed"; exit 1; }
timeout -k 10 120 python scripts/mfma_stats.py --variants 151,156 > gpurun_out/mfma_stats_t.json 2>&1 || { echo "stats failed"; exit 1; }
timeout -k 10 200 python scripts/ab_variants.py --config C --width 480 --height 270 --frames 2 --variants ${CVARIANTS:-152,154,155} --rounds 1 > gpurun_out/ab_C_t.json 2>&1 || { echo "ab C failed"; exit 1; }
echo "all ok"
