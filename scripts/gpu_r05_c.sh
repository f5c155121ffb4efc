#!/bin/bash
# round 5: tail-job debug (pixel diffs of 288/295/296 vs 282), resident kernel tests and A/B, every rank's
# slab, the tiled kernel with register fragments at 4 / 3 waves on a config C sample
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/debug_variants.py --config A --variants 282,295,296,288 > gpurun_out/r05c_debug_A.jsonl 2>&1
timeout -k 10 120 python -u scripts/debug_variants.py --config B --width 480 --height 270 --rays 8 --variants 282,295,296,288 > gpurun_out/r05c_debug_B.jsonl 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_filter_probe.py -x -q --timeout 120 --timeout-method thread -k "282 or 291 or 292 or 293 or 217 or 294" > gpurun_out/r05c_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config B --variants 282,284,294,263 --rounds 3 > gpurun_out/r05c_ab_B.json 2> gpurun_out/r05c_ab_B.err || exit 1
timeout -k 10 400 python -u scripts/shard_probe.py --config B --variants 282 --reps 2 > gpurun_out/r05c_shard_B.jsonl 2> gpurun_out/r05c_shard_B.err || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config C --width 480 --height 270 --frames 2 --variants 217,291,292,293 --rounds 3 > gpurun_out/r05c_ab_Cs.json 2> gpurun_out/r05c_ab_Cs.err
