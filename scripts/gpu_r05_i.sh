#!/bin/bash
# round 5: the resident kernel's split-half sweep for <= 32 live rays (308-311) and the packed path state
# without the record re-read (312): parity tests, config B A/B, every rank's slab
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_filter_probe.py -x -q --timeout 120 --timeout-method thread -k "308 or 309 or 310 or 311 or 312" > gpurun_out/r05i_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/ab_variants.py --config B --variants 282,308,309,310,311,312 --rounds 3 > gpurun_out/r05i_ab_B.json 2> gpurun_out/r05i_ab_B.err || exit 1
timeout -k 10 500 python -u scripts/shard_probe.py --config B --variants 282,308,311 --reps 2 > gpurun_out/r05i_shard_B.jsonl 2> gpurun_out/r05i_shard_B.err
