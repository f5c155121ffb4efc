#!/bin/bash
# round 5: the resident kernels with the per-segment wave maxima by DPP lane moves (306 = 282 + dpp,
# 307 = 298 + dpp): tests, config B A/B and slabs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RT2_LIB=exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 120 --timeout-method thread -k "v306 or v307" > gpurun_out/r05v_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/ab_variants.py --config B --variants 282,306 --rounds 5 > gpurun_out/r05v_ab_B.json 2> gpurun_out/r05v_ab_B.err || exit 1
timeout -k 10 500 python -u scripts/shard_probe.py --config B --variants 298,307 --ns 2,4,8 --reps 2 > gpurun_out/r05v_shard_B.jsonl 2> gpurun_out/r05v_shard_B.err
