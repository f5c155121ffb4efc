#!/bin/bash
# Y-by-matrix-product variant (150/151) and prefetch variants (148/149):
# parity tests on the experiment build, then interleaved A/B on config B,
# the matrix-filter counters and the rank-slab probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export RT2_LIB=exp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py -x -v --timeout 120 --timeout-method thread -k "${TESTK:-v150 or v151 or v148}" > gpurun_out/ymma_tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 240 python scripts/ab_variants.py --config B --variants ${VARIANTS:-140,150,148} --rounds 3 > gpurun_out/ab_B.json 2>&1 || { echo "ab B failed"; exit 1; }
timeout -k 10 120 python scripts/mfma_stats.py --variants 147,151 > gpurun_out/mfma_stats_y.json 2>&1 || { echo "stats failed"; exit 1; }
timeout -k 10 170 python scripts/shard_probe.py --variants ${SVARIANTS:-140,150} > gpurun_out/shard_ab.log 2>&1 || { echo "shard probe failed"; exit 1; }
echo "all ok"
