#!/bin/bash
# round 5: BVH v4 with the tree's top in LDS (treelet, variant 110): BVH parity tests, A/B on configs B, C, E
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bvh.py -x -q -k "111 or test_bvh2_large or big_leaves" --timeout 200 --timeout-method thread > gpurun_out/r05n_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config B --traversal bvh --variants 109,110,111 --rounds 3 > gpurun_out/r05n_ab_B.json 2> gpurun_out/r05n_ab_B.err || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config C --traversal bvh --variants 109,110,111 --rounds 3 > gpurun_out/r05n_ab_C.json 2> gpurun_out/r05n_ab_C.err || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config E --traversal bvh --variants 109,110,111 --rounds 3 > gpurun_out/r05n_ab_E.json 2> gpurun_out/r05n_ab_E.err
