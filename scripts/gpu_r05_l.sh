#!/bin/bash
# round 5: issue priority by rank within the SIMD (300; diag 301) against the quartile form (298), and the
# spread run order (RT2_RUN_ORDER=spread) on rank slabs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RT2_LIB=exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 120 --timeout-method thread -k "v300" > gpurun_out/r05l_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/mfma_timeline.py --wg-waves 16 --runs 299:8,301:8 > gpurun_out/r05l_timeline.jsonl 2> gpurun_out/r05l_timeline.err || exit 1
timeout -k 10 400 python -u scripts/ab_variants.py --config B --variants 282,298,300 --rounds 3 > gpurun_out/r05l_ab_B.json 2> gpurun_out/r05l_ab_B.err || exit 1
timeout -k 10 500 python -u scripts/shard_probe.py --config B --variants 282,298,300 --reps 2 > gpurun_out/r05l_shard_B.jsonl 2> gpurun_out/r05l_shard_B.err || exit 1
RT2_RUN_ORDER=spread timeout -k 10 500 python -u scripts/shard_probe.py --config B --variants 298,300 --reps 2 > gpurun_out/r05l_shard_B_spread.jsonl 2> gpurun_out/r05l_shard_B_spread.err || exit 1
RT2_RUN_ORDER=spread timeout -k 10 300 python -u scripts/mfma_timeline.py --wg-waves 16 --runs 299:8 > gpurun_out/r05l_timeline_spread.jsonl 2> gpurun_out/r05l_timeline_spread.err
