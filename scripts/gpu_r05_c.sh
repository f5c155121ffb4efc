#!/bin/bash
# round 5: resident kernel (thr_frag without branches, hoisted triangle pointer) with and without tail
# jobs; every rank's slab; the tiled kernel with register fragments at 4 / 3 waves on a config C sample
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_filter_probe.py -x -q --timeout 120 --timeout-method thread -k "282 or 288 or 291 or 217" > gpurun_out/r05c_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config B --variants 282,284,288,289,290,263 --rounds 3 > gpurun_out/r05c_ab_B.json 2> gpurun_out/r05c_ab_B.err || exit 1
timeout -k 10 400 python -u scripts/shard_probe.py --config B --variants 282,288 --reps 2 > gpurun_out/r05c_shard_B.jsonl 2> gpurun_out/r05c_shard_B.err || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config C --width 480 --height 270 --frames 2 --variants 217,291,292,293 --rounds 3 > gpurun_out/r05c_ab_Cs.json 2> gpurun_out/r05c_ab_Cs.err
