#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "brute_variants or split" > gpurun_out/t.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 400 python scripts/shard_probe.py --variants 85,90,91,85,90,91 > gpurun_out/shard.log 2>&1 || { echo "probe failed"; exit 1; }
echo "all ok"
