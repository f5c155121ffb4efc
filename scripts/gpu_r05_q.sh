#!/bin/bash
# round 5: two rays per lane at 2 waves per SIMD (303) and the hoisted threshold fragment (302):
# parity tests, config B A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RT2_LIB=exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_filter_probe.py -x -q --timeout 120 --timeout-method thread -k "302 or 303" > gpurun_out/r05q_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/ab_variants.py --config B --variants 282,302,303 --rounds 3 > gpurun_out/r05q_ab_B.json 2> gpurun_out/r05q_ab_B.err
