#!/bin/bash
# round 5: wave timelines of the resident kernel (diag builds 287, 297) and the longest-remaining-first issue
# priority (295, 296): parity tests, config B A/B, every rank's slab (experiment library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RT2_LIB=exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_filter_probe.py -x -q --timeout 120 --timeout-method thread -k "295 or 296" > gpurun_out/r05j_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/mfma_timeline.py --wg-waves 16 --runs 287:1,287:8,297:1,297:8 > gpurun_out/r05j_timeline.jsonl 2> gpurun_out/r05j_timeline.err || exit 1
timeout -k 10 400 python -u scripts/ab_variants.py --config B --variants 282,295,296 --rounds 3 > gpurun_out/r05j_ab_B.json 2> gpurun_out/r05j_ab_B.err || exit 1
timeout -k 10 500 python -u scripts/shard_probe.py --config B --variants 282,295,296 --reps 2 > gpurun_out/r05j_shard_B.jsonl 2> gpurun_out/r05j_shard_B.err
