#!/bin/bash
# round 5: resident kernel with records re-read per block (302, 303 + DPP maxima) and the packed path state
# (304): tests, A/B on config B, slabs, PMC of 304
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_filter_probe.py -x -q --timeout 120 --timeout-method thread -k "302 or 304" > gpurun_out/r05g_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config B --variants 282,302,303,304 --rounds 3 > gpurun_out/r05g_ab_B.json 2> gpurun_out/r05g_ab_B.err || exit 1
timeout -k 10 400 python -u scripts/shard_probe.py --config B --variants 304 --reps 2 > gpurun_out/r05g_shard_B.jsonl 2> gpurun_out/r05g_shard_B.err || exit 1
EXTRA_MFMA=1 EXTRA_L2=1 PMC_OUT=gpurun_out/r05g_pmc BENCH_ARGS="--variant 304" bash scripts/profile_pmc.sh > gpurun_out/r05g_pmc.log 2>&1
