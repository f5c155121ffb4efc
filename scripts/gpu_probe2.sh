#!/bin/bash
# Team tail modes on the slabs; tiled brute variants on config C (reduced spp).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/shard_probe.py --variants 85,64,65,66 > gpurun_out/shard_team.log 2>&1 || { echo "probe failed"; exit 1; }
timeout -k 10 300 python scripts/ab_variants.py --config C --rays 2 --frames 1 --variants 2,8,13,26 --rounds 2 > gpurun_out/ab_C.json 2>&1 || { echo "ab C failed"; exit 1; }
echo "all ok"
