#!/bin/bash
# round 5: the threshold fragment built once per sweep (302 = 282 + thr_hoist): tests, config B A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RT2_LIB=exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 120 --timeout-method thread -k "v302" > gpurun_out/r05p_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/ab_variants.py --config B --variants 282,302 --rounds 4 > gpurun_out/r05p_ab_B.json 2> gpurun_out/r05p_ab_B.err
