#!/bin/bash
# round 5: tail-job debugging (owner-only units; inlined unit), then the tiled kernel with register
# fragments (293) against 217 on full configs C and E
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/debug_variants.py --config A --variants 282,295,297,298 > gpurun_out/r05d_debug_A.jsonl 2>&1
timeout -k 10 120 python -u scripts/debug_variants.py --config B --width 480 --height 270 --rays 8 --variants 282,295,297,298 > gpurun_out/r05d_debug_B.jsonl 2>&1
timeout -k 10 600 python -u scripts/ab_variants.py --config C --variants 217,293 --rounds 2 > gpurun_out/r05d_ab_C.json 2> gpurun_out/r05d_ab_C.err || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py --config E --variants 217,293 --rounds 2 > gpurun_out/r05d_ab_E.json 2> gpurun_out/r05d_ab_E.err
