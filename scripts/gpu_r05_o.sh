#!/bin/bash
# round 5: where the tiled kernel's wave cycles go (diag build 305 of 293: shader clocks in the group filter,
# the exact phase and the tile waits) on a config C sample and full config E
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RT2_LIB=exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 120 --timeout-method thread -k "v306" > gpurun_out/r05o_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config C --width 480 --height 270 --rays 64 --variants 293,305,306,307 --rounds 2 > gpurun_out/r05o_ab_Cs.json 2> gpurun_out/r05o_ab_Cs.err || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config E --variants 293,305,306,307 --rounds 1 > gpurun_out/r05o_ab_E.json 2> gpurun_out/r05o_ab_E.err
