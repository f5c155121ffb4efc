#!/bin/bash
# Round 3: the whole GPU suite (probe summary to gpurun_out/filter_probe.json) and smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
RT2_PROBE_OUT=gpurun_out/filter_probe.json timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
if [ -n "${REHEARSE}" ]; then
  RT2_BENCH_BACKEND=gloo timeout -k 10 240 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/rehearse_B.log 2>&1 || { echo "2-rank rehearsal failed"; exit 1; }
fi
echo "all ok"
