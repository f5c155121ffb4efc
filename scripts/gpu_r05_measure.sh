#!/bin/bash
# Round 5 measurement call (stages by environment flag; each stops the script on failure):
#   TESTS=1     GPU suite + smoke
#   BENCH=1     the default bench line (config B + the C / E / scalar-VALU legs, CPU baseline)
#   STATS="B C" rocprofv3 --kernel-trace --stats of a bench run per config (per-kernel averages, csv)
#   PMC_CONFIGS PMC passes (scripts/profile_pmc.sh) of the bench's render kernel per config ("B C E")
#   SHARD="B D" every rank's slab on one GPU (scripts/shard_probe.py), automatic kernel
# Summaries: python scripts/parse_pmc.py <config> with PMC_DIR=gpurun_out/pmc<config> (CPU side).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${TESTS}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
fi
if [ -n "${BENCH}" ]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
  echo "bench ok"
fi
for c in ${STATS}; do
  case $c in
    B) a="" ; d=stats ;;
    *) a="--config $c --steps 1 --warmup 0" ; d=stats$c ;;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$d -o run -- python3 bench.py --no-cpu-baseline --no-config-c --no-config-e --no-scalar --no-alt $a > gpurun_out/$d.log 2>&1 || { echo "stats $c failed"; tail -20 gpurun_out/$d.log; exit 1; }
  echo "stats $c ok"
done
for c in ${PMC_CONFIGS}; do
  case $c in
    B) a="" ;;
    *) a="--config $c --steps 1 --warmup 0" ;;
  esac
  PMC_OUT=gpurun_out/pmc$c BENCH_ARGS="$a" EXTRA_MFMA=1 EXTRA_L2=1 bash scripts/profile_pmc.sh > gpurun_out/pmc$c.out 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc$c.out; exit 1; }
  echo "pmc $c ok"
done
for c in ${SHARD}; do
  timeout -k 10 500 python -u scripts/shard_probe.py --config $c --reps 1 > gpurun_out/shard_probe_$c.jsonl 2> gpurun_out/shard_probe_$c.err || { echo "shard probe $c failed"; tail -20 gpurun_out/shard_probe_$c.err; exit 1; }
  echo "shard probe $c ok"
done
echo "all ok"
