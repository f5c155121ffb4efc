#!/bin/bash
# Round 4 GPU runner: each stage runs only when its variable is set, under its
# own time limit, and the script stops at the first failure.
#   TESTS=1            the whole GPU suite (PYTEST_ARGS extra args) + smoke()
#   PYTEST_K=expr      only tests/test_gpu_mfma.py -k expr
#   VARIANTS=a,b       interleaved A/B on config B (ROUNDS, default 3)
#   CVARIANTS=a,b      A/B on a config C sample (480x270, 2 frames)
#   CFULL=a,b          A/B on the full config C step (1920x1080, 256 spp), 1 round
#   EVARIANTS=a,b      A/B on a config E sample (480x270, 4 spp)
#   EFULL=a,b          A/B on the full config E step (1920x1080, 4 spp), 1 round
#   SVARIANTS=a,b      rank-slab probe of config B (scripts/shard_probe.py)
#   BENCH=1            python bench.py (BENCH_ARGS)
#   AB_LIB=exp         the A/B stages load the experiment build (rt2/librt2_exp.so)
#   SHARD_D=v          rank-slab probe of config D (4K, 1,024 spp) with variant v (0 = automatic)
#   STATS=1            rocprofv3 --kernel-trace --stats of the default bench workload
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "${TESTS}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
if [ -n "${PYTEST_K}" ]; then
  RT2_LIB=${AB_LIB:-$RT2_LIB} timeout -k 10 500 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_filter_probe.py -x -v --timeout 150 --timeout-method thread -k "${PYTEST_K}" > gpurun_out/mfma_tests.log 2>&1 || { echo "mfma tests failed"; tail -30 gpurun_out/mfma_tests.log; exit 1; }
  tail -2 gpurun_out/mfma_tests.log
fi
if [ -n "${VARIANTS}" ]; then
  RT2_LIB=${AB_LIB:-$RT2_LIB} timeout -k 10 300 python scripts/ab_variants.py --config B --variants ${VARIANTS} --rounds ${ROUNDS:-3} > gpurun_out/ab_B.json 2>&1 || { echo "ab B failed"; tail -20 gpurun_out/ab_B.json; exit 1; }
fi
if [ -n "${CVARIANTS}" ]; then
  RT2_LIB=${AB_LIB:-$RT2_LIB} timeout -k 10 300 python scripts/ab_variants.py --config C --width 480 --height 270 --frames 2 --variants ${CVARIANTS} --rounds 2 > gpurun_out/ab_C.json 2>&1 || { echo "ab C failed"; tail -20 gpurun_out/ab_C.json; exit 1; }
fi
if [ -n "${EVARIANTS}" ]; then
  RT2_LIB=${AB_LIB:-$RT2_LIB} timeout -k 10 400 python scripts/ab_variants.py --config E --width 480 --height 270 --rays 4 --variants ${EVARIANTS} --rounds 2 > gpurun_out/ab_E.json 2>&1 || { echo "ab E failed"; tail -20 gpurun_out/ab_E.json; exit 1; }
fi
if [ -n "${EFULL}" ]; then
  RT2_LIB=${AB_LIB:-$RT2_LIB} timeout -k 10 400 python scripts/ab_variants.py --config E --variants ${EFULL} --rounds 1 > gpurun_out/ab_Efull.json 2>&1 || { echo "ab E full failed"; tail -20 gpurun_out/ab_Efull.json; exit 1; }
fi
if [ -n "${CFULL}" ]; then
  RT2_LIB=${AB_LIB:-$RT2_LIB} timeout -k 10 500 python scripts/ab_variants.py --config C --variants ${CFULL} --rounds 1 > gpurun_out/ab_Cfull.json 2>&1 || { echo "ab C full failed"; tail -20 gpurun_out/ab_Cfull.json; exit 1; }
fi
if [ -n "${SVARIANTS}" ]; then
  RT2_LIB=${AB_LIB:-$RT2_LIB} timeout -k 10 300 python scripts/shard_probe.py --reps ${SREPS:-3} --variants ${SVARIANTS} > gpurun_out/shard_ab.log 2>&1 || { echo "shard probe failed"; tail -20 gpurun_out/shard_ab.log; exit 1; }
fi
if [ -n "${SHARD_D}" ]; then
  timeout -k 10 400 python scripts/shard_probe.py --config D --reps 1 --variants ${SHARD_D} > gpurun_out/shard_probe_D.log 2>&1 || { echo "shard probe D failed"; tail -20 gpurun_out/shard_probe_D.log; exit 1; }
fi
if [ -n "${STATS}" ]; then
  # rocprofv3 kernel-trace summary of the default bench workload (config B)
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats -o run -- python3 bench.py --no-cpu-baseline --no-alt --no-config-c --no-config-e --no-scalar --steps 5 --warmup 2 > gpurun_out/stats_bench.log 2>&1 || { echo "rocprof stats failed"; tail -20 gpurun_out/stats_bench.log; exit 1; }
fi
if [ -n "${BENCH}" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
fi
echo "all ok"
