#!/bin/bash
# plk filter: GPU parity of the new variants, then interleaved A/B on config B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "plk or brute_variants" > gpurun_out/gpu_plk_tests.log 2>&1 || { echo "plk tests failed"; exit 1; }
timeout -k 10 240 python scripts/ab_variants.py --variants 0,90,91,0,90,91 --rounds 2 > gpurun_out/ab_plk.json 2>&1 || { echo "ab failed"; exit 1; }
echo "all ok"
