#!/bin/bash
# Round 3: config E (1M triangles) bench line (brute force = the k16 matrix kernel,
# BVH beside it, CPU baseline) + its kernel trace; PMC passes of config C's
# brute-force (full size, one launch per pass) and BVH launches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_E}" ]; then
  timeout -k 10 600 python bench.py --config E --steps 1 --warmup 0 --cpu-seconds 10 > gpurun_out/bench_E.log 2>&1 || { echo "bench E failed"; exit 1; }
fi
if [ -n "${PMC_C}" ]; then
  mkdir -p gpurun_out/pmcC && rm -rf gpurun_out/pmc_*
  BENCH_ARGS="--config C --steps 1 --warmup 0" EXTRA_MFMA=1 EXTRA_L2=1 bash scripts/profile_pmc.sh > gpurun_out/pmc.log 2>&1 || { echo "pmc C failed"; exit 1; }
  mv gpurun_out/pmc_* gpurun_out/pmcC/
  BENCH_ARGS="--config C --traversal bvh --steps 2 --warmup 1" EXTRA_L2=1 bash scripts/profile_pmc.sh > gpurun_out/pmc_bvh.log 2>&1 || { echo "pmc C bvh failed"; exit 1; }
fi
echo "all ok"
