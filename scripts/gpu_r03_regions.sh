#!/bin/bash
# Round 3: item regions (XCD-group bands) vs one dispatch-order counter for the
# brute-force kernel: rank-slab probe under both policies, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/regions.log
for pass in 1 2; do
  RT2_ITEM_REGIONS=1 timeout -k 10 200 python scripts/shard_probe.py --variants 0 >> gpurun_out/regions.log 2>&1 || { echo "probe (regions) failed"; exit 1; }
  RT2_ITEM_REGIONS=0 timeout -k 10 200 python scripts/shard_probe.py --variants 0 >> gpurun_out/regions.log 2>&1 || { echo "probe (one counter) failed"; exit 1; }
done
echo "all ok"
