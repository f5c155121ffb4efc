#!/bin/bash
# Slab probe with and without most-expensive-first item order.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/shard_probe.py --variants 0 --cost-order 0 > gpurun_out/shard_co0.log 2>&1 || { echo "probe failed"; exit 1; }
timeout -k 10 300 python scripts/shard_probe.py --variants 0 --cost-order 1 > gpurun_out/shard_co1.log 2>&1 || { echo "probe failed"; exit 1; }
echo "all ok"
