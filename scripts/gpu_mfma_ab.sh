#!/bin/bash
# Matrix-filter kernel: its GPU parity tests and the launcher tests, then
# interleaved same-process A/B of VARIANTS on config B, a config C sample
# (CVARIANTS) and the rank-slab probe (SVARIANTS).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "mfma or auto_variant or split_waves or brute_variants" > gpurun_out/mfma_tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 240 python scripts/ab_variants.py --config B --variants ${VARIANTS:-0,131} --rounds 3 > gpurun_out/ab_B.json 2>&1 || { echo "ab B failed"; exit 1; }
if [ -n "${CVARIANTS}" ]; then
  timeout -k 10 170 python scripts/ab_variants.py --config C --width 480 --height 270 --frames 2 --variants ${CVARIANTS} --rounds 2 > gpurun_out/ab_C.json 2>&1 || { echo "ab C failed"; exit 1; }
fi
if [ -n "${SVARIANTS}" ]; then
  timeout -k 10 170 python scripts/shard_probe.py --variants ${SVARIANTS} > gpurun_out/shard_ab.log 2>&1 || { echo "shard probe failed"; exit 1; }
fi
echo "all ok"
