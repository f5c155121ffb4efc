#!/bin/bash
# Round 3: the filter probe + near-threshold scene, the k16 sweep's parity
# tests, then interleaved A/B of the matrix-filter variants on config B and a
# config C sample.  Each GPU step has its own limit; the chain stops at the
# first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
RT2_PROBE_OUT=gpurun_out/filter_probe.json timeout -k 10 300 python -u -m pytest tests/test_gpu_filter_probe.py -x -v --timeout 150 --timeout-method thread > gpurun_out/probe_tests.log 2>&1 || { echo "probe tests failed"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfma.py -x -v --timeout 150 --timeout-method thread > gpurun_out/mfma_tests.log 2>&1 || { echo "mfma tests failed"; exit 1; }
timeout -k 10 240 python scripts/ab_variants.py --config B --variants ${VARIANTS:-152,160,161,162,163,164,166,167,168} --rounds 3 > gpurun_out/ab_B.json 2>&1 || { echo "ab B failed"; exit 1; }
timeout -k 10 240 python scripts/ab_variants.py --config C --width 480 --height 270 --frames 2 --variants ${CVARIANTS:-150,160,162,164,168} --rounds 2 > gpurun_out/ab_C.json 2>&1 || { echo "ab C failed"; exit 1; }
echo "all ok"
