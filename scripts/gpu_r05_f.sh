#!/bin/bash
# round 5: tail jobs served by helpers only (owners wait): correctness, whole-image A/B, every rank's slab
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/debug_variants.py --config A --variants 282,288,289,290 > gpurun_out/r05f_debug_A.jsonl 2>&1
timeout -k 10 120 python -u scripts/debug_variants.py --config B --width 480 --height 270 --rays 8 --variants 282,288,289,290 > gpurun_out/r05f_debug_B.jsonl 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_filter_probe.py -x -q --timeout 120 --timeout-method thread -k "288 or 289" > gpurun_out/r05f_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config B --variants 282,288,289,290 --rounds 3 > gpurun_out/r05f_ab_B.json 2> gpurun_out/r05f_ab_B.err || exit 1
timeout -k 10 400 python -u scripts/shard_probe.py --config B --variants 282,288,289 --reps 2 > gpurun_out/r05f_shard_B.jsonl 2> gpurun_out/r05f_shard_B.err
