#!/bin/bash
# PMC passes over an arbitrary python command (one counter group per
# rocprofv3 run, --pmc only; no sys/runtime trace).  Usage:
#   scripts/pmc_probe.sh <tag> <python args...>
# Output: gpurun_out/pmcp_<tag>_<group>/ and .log
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1
shift
run() {
  local name=$1
  local counters=$2
  shift 2
  timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcp_${TAG}_$name" -o run \
    -- python3 "$@" > "$GRAFT_REPO_ROOT/gpurun_out/pmcp_${TAG}_$name.log" 2>&1
}
ARGS=("$@")
run valu "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "${ARGS[@]}" && \
run thread "SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "${ARGS[@]}" && \
run wait "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD" "${ARGS[@]}" && \
run l2 "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "${ARGS[@]}" && \
run fetch "FETCH_SIZE" "${ARGS[@]}" && \
echo "pmc ok"
