#!/bin/bash
# Round 3, session 2: the MFMA/VALU overlap micro-probe (scripts/overlap_probe.hip),
# the k16 wave timeline with in-kernel clocks, and 2-wave builds on the rank slabs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/overlap_probe ${PROBE_ITERS:-20000} > gpurun_out/overlap_probe.log 2>&1 || { echo "overlap probe failed"; exit 1; }
export RT2_LIB=exp
timeout -k 10 200 python scripts/mfma_timeline.py --runs "${TL_RUNS:-210:1,222:8}" > gpurun_out/timeline2.log 2>&1 || { echo "timeline failed"; exit 1; }
timeout -k 10 300 python scripts/shard_probe.py --variants "${SHARD_VARIANTS:-0,212,199}" > gpurun_out/shard_w2.log 2>&1 || { echo "shard w2 failed"; exit 1; }
echo "all ok"
