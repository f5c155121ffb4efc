#!/bin/bash
# Round 3: experiment-build A/B (RT2_LIB=exp): parity tests of the chosen
# experiment variants, then interleaved A/B on config B, a config C sample and
# the rank-slab probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export RT2_LIB=exp
if [ -n "${PYTEST_K}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_mfma.py -x -v --timeout 150 --timeout-method thread -k "${PYTEST_K}" > gpurun_out/mfma_tests.log 2>&1 || { echo "mfma tests failed"; exit 1; }
fi
timeout -k 10 240 python scripts/ab_variants.py --config B ${DUP:+--dup $DUP} --no-check "${NOCHECK}" --variants ${VARIANTS} --rounds ${ROUNDS:-3} > gpurun_out/ab_B.json 2>&1 || { echo "ab B failed"; exit 1; }
if [ -n "${CVARIANTS}" ]; then
  timeout -k 10 300 python scripts/ab_variants.py --config C --width 480 --height 270 --frames 2 --no-check "${NOCHECK}" --variants ${CVARIANTS} --rounds 2 > gpurun_out/ab_C.json 2>&1 || { echo "ab C failed"; exit 1; }
fi
if [ -n "${SVARIANTS}" ]; then
  timeout -k 10 200 python scripts/shard_probe.py --variants ${SVARIANTS} > gpurun_out/shard_ab.log 2>&1 || { echo "shard probe failed"; exit 1; }
fi
echo "all ok"
