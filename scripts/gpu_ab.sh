#!/bin/bash
# Brute-variant parity on the GPU, then an interleaved same-process A/B of
# VARIANTS (comma list) on config B (CONFIG to change it).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "plk or brute_variants or split or auto_variant" > gpurun_out/gpu_ab_tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python scripts/ab_variants.py --config ${CONFIG:-B} --variants ${VARIANTS:-0,28} --rounds ${ROUNDS:-3} > gpurun_out/ab.json 2>&1 || { echo "ab failed"; exit 1; }
echo "all ok"
