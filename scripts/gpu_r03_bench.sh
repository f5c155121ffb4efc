#!/bin/bash
# Round 3: default bench (config B headline + BVH + CPU baseline + config C legs),
# the rocprofv3 kernel trace of the headline, the PMC passes of config B's render
# kernel and the rank-slab probe.  Each GPU step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
{ grep -m1 "model name" /proc/cpuinfo; nproc; cat /sys/fs/cgroup/cpu.max; } > gpurun_out/host.txt 2>&1
if [ -z "${SKIP_BENCH}" ]; then
  timeout -k 10 480 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; exit 1; }
fi
export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-alt --no-config-c > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed"; exit 1; }
if [ -n "${PMC}" ]; then
  EXTRA_MFMA=1 EXTRA_L2=1 bash scripts/profile_pmc.sh > gpurun_out/pmc.log 2>&1 || { echo "pmc failed"; exit 1; }
fi
timeout -k 10 150 python scripts/shard_probe.py --variants 0 > gpurun_out/shard.log 2>&1 || { echo "shard probe failed"; exit 1; }
echo "all ok"
