#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof kernel trace, shard-slab probe,
# config D 2-rank rehearsal.  Every GPU step has its own time limit and the
# chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
{ grep -m1 "model name" /proc/cpuinfo; nproc; cat /sys/fs/cgroup/cpu.max; } > gpurun_out/host.txt 2>&1
timeout -k 10 360 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 420 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; exit 1; }
if [ -n "${SHARD_PROBE}" ]; then
  timeout -k 10 120 python scripts/shard_probe.py --variants ${SHARD_VARIANTS:-0} > gpurun_out/shard.log 2>&1 || { echo "shard probe failed"; exit 1; }
fi
if [ -n "${REHEARSE_D}" ]; then
  RT2_BENCH_BACKEND=gloo timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config D --steps 1 --warmup 0 \
    --no-cpu-baseline --no-alt > gpurun_out/rehearse_D.log 2>&1 || { echo "config D rehearsal failed"; exit 1; }
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-alt --no-config-c ${BENCH_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed"; exit 1; }
echo "all ok"
