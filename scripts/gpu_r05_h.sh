#!/bin/bash
# round 5: tiled kernel with records re-read per block (306) and the single-pass Y reduction (305):
# parity tests, config C (sample + full) and E A/B against 293
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_filter_probe.py -x -q --timeout 120 --timeout-method thread -k "305 or 306" > gpurun_out/r05h_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config C --width 480 --height 270 --rays 64 --variants 293,305,306 --rounds 3 > gpurun_out/r05h_ab_Cs.json 2> gpurun_out/r05h_ab_Cs.err || exit 1
timeout -k 10 400 python -u scripts/ab_variants.py --config E --variants 293,305,306 --rounds 2 > gpurun_out/r05h_ab_E.json 2> gpurun_out/r05h_ab_E.err || exit 1
timeout -k 10 700 python -u scripts/ab_variants.py --config C --variants 293,305 --rounds 1 > gpurun_out/r05h_ab_C.json 2> gpurun_out/r05h_ab_C.err
