#!/bin/bash
# Shard-slab probe for a list of variants (VARIANTS), config B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python scripts/shard_probe.py --variants ${VARIANTS:-0,28} > gpurun_out/shard.log 2>&1 || { echo "probe failed"; exit 1; }
echo "all ok"
