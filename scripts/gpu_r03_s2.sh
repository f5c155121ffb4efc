#!/bin/bash
# Round 3, session 2: GPU suite + smoke + default bench + rocprof (scripts/gpu_r03_tests.sh,
# gpu_r03_bench.sh), then the k16 wave timeline (diag variants) and the lockstep vs
# free-running A/B on config B (whole image and rank slabs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "${SKIP_BASE}" ]; then
  bash scripts/gpu_r03_tests.sh || exit 1
  BENCH_ARGS="${BENCH_ARGS:---steps 5 --warmup 2}" bash scripts/gpu_r03_bench.sh || exit 1
fi
export RT2_LIB=exp
timeout -k 10 200 python scripts/mfma_timeline.py --runs "${TL_RUNS:-210:1,222:8,210:8,225:1,226:8}" > gpurun_out/timeline.log 2>&1 || { echo "timeline failed"; exit 1; }
timeout -k 10 300 python scripts/ab_variants.py --variants "${AB_VARIANTS:-200,223}" --rounds 3 > gpurun_out/ab_free.log 2>&1 || { echo "ab failed"; exit 1; }
timeout -k 10 300 python scripts/shard_probe.py --variants "${SHARD_VARIANTS:-0,223,206,224}" > gpurun_out/shard_free.log 2>&1 || { echo "shard ab failed"; exit 1; }
echo "all ok"
