#!/bin/bash
# round 5: first look at the LDS-resident small-scene kernel (variants 280-283) vs 263
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_filter_probe.py -x -q --timeout 120 --timeout-method thread -k "v280 or v281 or v282 or v283 or v263 or 280 or 281 or 282 or 283 or 263" > gpurun_out/r05a_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config B --variants 263,280,281,282,283 --rounds 3 > gpurun_out/r05a_ab_B.json 2> gpurun_out/r05a_ab_B.err
