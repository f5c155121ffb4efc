#!/bin/bash
# round 5: triple-buffered record tiles with register fragments (306: 12 groups x 3, 307: 9 groups x 3):
# two tiles of LDS-DMA lead instead of one; tests, config C sample and E A/B against 293
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RT2_LIB=exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 120 --timeout-method thread -k "v306 or v307" > gpurun_out/r05t_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config C --width 480 --height 270 --rays 64 --variants 293,306,307 --rounds 3 > gpurun_out/r05t_ab_Cs.json 2> gpurun_out/r05t_ab_Cs.err || exit 1
timeout -k 10 400 python -u scripts/ab_variants.py --config E --variants 293,306,307 --rounds 2 > gpurun_out/r05t_ab_E.json 2> gpurun_out/r05t_ab_E.err
