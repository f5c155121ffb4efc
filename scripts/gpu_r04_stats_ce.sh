#!/bin/bash
# rocprofv3 kernel-trace summaries of the config C and E bench legs (one
# brute-force step each, no CPU baseline), for profiles/r04_config{C,E}_kernel_stats.csv
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in C E; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats$c -o run -- python3 bench.py --config $c --no-cpu-baseline --no-alt --no-scalar --steps 1 --warmup 0 > gpurun_out/stats$c.log 2>&1 || { echo "stats $c failed"; tail -5 gpurun_out/stats$c.log; exit 1; }
  echo "stats $c ok"
done
