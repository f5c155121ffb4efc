#!/bin/bash
# Matrix-filter kernel: its GPU parity tests, then interleaved A/B against the
# scalar-path default on config B and a config C frame sample.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_mfma.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mfma_tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 240 python scripts/ab_variants.py --config B --variants ${VARIANTS:-0,130,131,132,133,134,135} --rounds 3 > gpurun_out/ab_B.json 2>&1 || { echo "ab B failed"; exit 1; }
echo "all ok"
