#!/bin/bash
# PMC passes for the brute-force kernel: scalar-cache behaviour, lane
# utilisation, issue mix (one counter group per rocprofv3 run, --pmc only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-brute}
run() {
  local name=$1
  local counters=$2
  timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcp_${TAG}_$name" -o run \
    -- python3 "$GRAFT_REPO_ROOT/scripts/ab_variants.py" --variants ${VARIANT:-0} --rounds 1 \
    > "$GRAFT_REPO_ROOT/gpurun_out/pmcp_${TAG}_$name.log" 2>&1
}
run sqc "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_TC_STALL" && \
run lane "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH" && \
run lvl "SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" && \
run cyc "SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES" && \
echo "pmc ok"
