#!/bin/bash
# Round 4 measurement call: GPU suite (TESTS=1), the default bench line, then
# PMC passes (scripts/profile_pmc.sh) of the bench's render kernel for the
# configurations in PMC_CONFIGS (e.g. "B C"); each stage stops the script on
# failure.  Summaries: python scripts/parse_pmc.py <config> with
# PMC_DIR=gpurun_out/pmc<config> (run on the CPU side afterwards).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
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
for c in ${PMC_CONFIGS}; do
  case $c in
    B) a="" ;;
    *) a="--config $c --steps 1 --warmup 0" ;;
  esac
  PMC_OUT=gpurun_out/pmc$c BENCH_ARGS="$a" EXTRA_MFMA=1 EXTRA_L2=1 bash scripts/profile_pmc.sh > gpurun_out/pmc$c.out 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc$c.out; exit 1; }
  echo "pmc $c ok"
done
if [ -n "${SHARD_D}" ]; then
  timeout -k 10 400 python scripts/shard_probe.py --config D --reps 1 > gpurun_out/shard_probe_D.log 2>&1 || { echo "shard probe D failed"; tail -20 gpurun_out/shard_probe_D.log; exit 1; }
  echo "shard probe D ok"
fi
echo "all ok"
