#!/bin/bash
# The one GPU-session runner (gpurun -- bash scripts/gpu_run.sh).  Stages are
# chosen by environment variables; each GPU step has its own time limit and
# the script stops at the first failure (no retries).
#   LIB=exp          use rt2/librt2_exp.so (the A/B experiment variants)
#   TESTS="<args>"   pytest -m gpu with these extra arguments ("all" = the whole suite, + smoke);
#   TESTK="<expr>"   ... and this -k expression
#   AB="<cfg>:<variants>[:<rounds>[:<extra>]] ..."
#                    interleaved A/B (scripts/ab_variants.py), identical images required;
#                    e.g. AB="B:282,320:5 C:293,330:1:--width 480 --height 270 --frames 2"
#   STATSV="<cfg>:<variants> ..."   diagnostic counters (scripts/mfma_stats.py)
#   SHARD="<cfg>[:<variants>] ..."  every rank's slab on one GPU (scripts/shard_probe.py)
#   BENCH="<args>"   python bench.py <args> -> gpurun_out/bench<TAG>.json ("default" = no args)
#   STATS="B C E"    rocprofv3 --kernel-trace --stats of a bench run per config
#   PMC="B C E"      PMC passes (scripts/profile_pmc.sh) of the bench's render kernel per config
#   TAG=<name>       suffix of the output files
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
[ -n "${LIB}" ] && export RT2_LIB=${LIB}
T=${TAG:-run}
mkdir -p gpurun_out
{ grep -m1 "model name" /proc/cpuinfo; nproc; cat /sys/fs/cgroup/cpu.max; } > gpurun_out/host_$T.txt 2>&1
if [ -n "${TESTS}" ]; then
  targs="${TESTS}"; [ "${TESTS}" = all ] && targs=""
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${targs} ${TESTK:+-k "$TESTK"} \
    > gpurun_out/gpu_tests_$T.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests_$T.log; exit 1; }
  tail -1 gpurun_out/gpu_tests_$T.log
  if [ "${TESTS}" = all ]; then
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { echo "smoke failed"; exit 1; }
  fi
fi
for spec in ${AB}; do
  IFS=: read -r cfg vars rounds extra <<< "${spec//+/ }"
  timeout -k 10 900 python -u scripts/ab_variants.py --config "$cfg" --variants "$vars" --rounds "${rounds:-3}" ${extra} \
    > "gpurun_out/ab_${T}_${cfg}.json" 2> "gpurun_out/ab_${T}_${cfg}.err" || { echo "A/B $spec failed"; tail -20 "gpurun_out/ab_${T}_${cfg}.err"; exit 1; }
  echo "A/B $cfg ok"; cat "gpurun_out/ab_${T}_${cfg}.json" | head -c 3000; echo
done
for spec in ${STATSV}; do
  IFS=: read -r cfg vars extra <<< "${spec//+/ }"
  timeout -k 10 600 python -u scripts/mfma_stats.py --config "$cfg" --variants "$vars" ${extra} \
    > "gpurun_out/mfma_stats_${T}_${cfg}.json" 2> "gpurun_out/mfma_stats_${T}_${cfg}.err" || { echo "stats $spec failed"; tail -20 "gpurun_out/mfma_stats_${T}_${cfg}.err"; exit 1; }
  cat "gpurun_out/mfma_stats_${T}_${cfg}.json"
done
for spec in ${SHARD}; do
  IFS=: read -r cfg vars <<< "$spec"
  va=""; [ -n "$vars" ] && va="--variants $vars"
  timeout -k 10 600 python -u scripts/shard_probe.py --config "$cfg" --reps 1 $va > "gpurun_out/shard_${T}_${cfg}.jsonl" \
    2> "gpurun_out/shard_${T}_${cfg}.err" || { echo "shard probe $spec failed"; tail -20 "gpurun_out/shard_${T}_${cfg}.err"; exit 1; }
  echo "shard probe $cfg ok"
done
if [ -n "${BENCH}" ]; then
  bargs="${BENCH}"; [ "${BENCH}" = default ] && bargs=""
  timeout -k 10 900 python bench.py ${bargs} > "gpurun_out/bench_$T.json" 2> "gpurun_out/bench_$T.err" \
    || { echo "bench failed"; tail -20 "gpurun_out/bench_$T.err"; exit 1; }
  echo "bench ok"; cut -c1-600 "gpurun_out/bench_$T.json"
fi
for c in ${STATS}; do
  case $c in
    B) a="" ;;
    *) a="--config $c --steps 1 --warmup 0" ;;
  esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/stats_${T}_$c" -o run -- \
    python3 bench.py --no-cpu-baseline --no-config-c --no-config-e --no-config-w --no-scalar --no-alt $a > "gpurun_out/stats_${T}_$c.log" 2>&1 \
    || { echo "stats $c failed"; tail -20 "gpurun_out/stats_${T}_$c.log"; exit 1; }
  echo "stats $c ok"
done
for c in ${PMC}; do
  case $c in
    B) a="" ;;
    *) a="--config $c --steps 1 --warmup 0" ;;
  esac
  PMC_OUT="gpurun_out/pmc_${T}_$c" BENCH_ARGS="$a" EXTRA_MFMA=1 EXTRA_L2=1 bash scripts/profile_pmc.sh > "gpurun_out/pmc_${T}_$c.out" 2>&1 \
    || { echo "pmc $c failed"; tail -5 "gpurun_out/pmc_${T}_$c.out"; exit 1; }
  echo "pmc $c ok"
done
echo "all ok"
