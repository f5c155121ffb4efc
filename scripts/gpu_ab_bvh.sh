#!/bin/bash
# GPU parity (brute + BVH) then A/B: brute default and BVH default on config B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 200 python scripts/ab_variants.py --variants 0,28 --rounds 3 > gpurun_out/ab_brute.json 2>&1 || { echo "ab failed"; exit 1; }
timeout -k 10 200 python scripts/ab_variants.py --traversal bvh --variants 53 --rounds 3 > gpurun_out/ab_bvh.json 2>&1 || { echo "ab bvh failed"; exit 1; }
echo "all ok"
