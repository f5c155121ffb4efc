#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/debug_variants.py --config A --variants 282,300,301,288 > gpurun_out/r05e2_debug_A.jsonl 2>&1
timeout -k 10 120 python -u scripts/debug_variants.py --config B --width 480 --height 270 --rays 8 --variants 282,300,301,288 > gpurun_out/r05e2_debug_B.jsonl 2>&1
