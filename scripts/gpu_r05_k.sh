#!/bin/bash
# round 5: fair-share issue priority on the resident kernel (298; diag 299): tests, timelines, A/B, slabs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RT2_LIB=exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 120 --timeout-method thread -k "v298" > gpurun_out/r05k_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/mfma_timeline.py --wg-waves 16 --runs 287:8,299:8,299:1 > gpurun_out/r05k_timeline.jsonl 2> gpurun_out/r05k_timeline.err || exit 1
timeout -k 10 400 python -u scripts/ab_variants.py --config B --variants 282,298 --rounds 3 > gpurun_out/r05k_ab_B.json 2> gpurun_out/r05k_ab_B.err || exit 1
timeout -k 10 500 python -u scripts/shard_probe.py --config B --variants 282,298 --reps 2 > gpurun_out/r05k_shard_B.jsonl 2> gpurun_out/r05k_shard_B.err
