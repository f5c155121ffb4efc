#!/bin/bash
# round 5: the Y product skipped for 32-ray blocks without a distance bound (y_skip: 302 = 282 + ysk,
# 303 = 298 + ysk, 304 = 293 + ysk): parity tests, config B A/B and slabs, config C sample and E A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RT2_LIB=exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_filter_probe.py -x -q --timeout 120 --timeout-method thread -k "302 or 303 or 304" > gpurun_out/r05m_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/ab_variants.py --config B --variants 282,302 --rounds 3 > gpurun_out/r05m_ab_B.json 2> gpurun_out/r05m_ab_B.err || exit 1
timeout -k 10 400 python -u scripts/shard_probe.py --config B --variants 298,303 --reps 2 > gpurun_out/r05m_shard_B.jsonl 2> gpurun_out/r05m_shard_B.err || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config C --width 480 --height 270 --rays 64 --variants 293,304 --rounds 3 > gpurun_out/r05m_ab_Cs.json 2> gpurun_out/r05m_ab_Cs.err || exit 1
timeout -k 10 400 python -u scripts/ab_variants.py --config E --variants 293,304 --rounds 2 > gpurun_out/r05m_ab_E.json 2> gpurun_out/r05m_ab_E.err
