#!/bin/bash
# round 5: the resident kernel with the threshold fragment hoisted (302), the exact phase's next-candidate
# prefetch (303) and both (304): parity tests, config B A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RT2_LIB=exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_filter_probe.py -x -q --timeout 120 --timeout-method thread -k "302 or 303 or 304" > gpurun_out/r05s_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u scripts/ab_variants.py --config B --variants 282,302,303,304 --rounds 4 > gpurun_out/r05s_ab_B.json 2> gpurun_out/r05s_ab_B.err
