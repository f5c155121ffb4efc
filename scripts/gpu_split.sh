#!/bin/bash
# Parity of the brute variants (incl. split-wave), then the shard-scaling probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "plk or brute_variants or split" > gpurun_out/t.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python scripts/shard_probe.py --variants ${VARIANTS:-0,71,83,84,85} > gpurun_out/shard.log 2>&1 || { echo "probe failed"; exit 1; }
echo "all ok"
