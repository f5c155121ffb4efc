#!/bin/bash
# PMC passes for the bench's render kernel (one counter group per rocprofv3 run,
# --kernel-trace/--pmc only; no sys/runtime trace).  Output: ${PMC_OUT:-gpurun_out}/pmc_<name>/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-alt --no-config-c --no-config-e --no-config-w --no-scalar --steps 2 --warmup 1 ${BENCH_ARGS}"
OUTD="$GRAFT_REPO_ROOT/${PMC_OUT:-gpurun_out}"
mkdir -p "$OUTD"
run() {
  local name=$1; shift
  local kt=""
  [ "$name" = clock ] && kt="--kernel-trace"  # kernel durations for the clock (GRBM_GUI_ACTIVE / 8 / ns)
  timeout -k 10 300 rocprofv3 $kt --pmc "$@" --output-format csv -d "$OUTD/pmc_$name" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$OUTD/pmc_$name.log" 2>&1
}
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
run salu SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES && \
run clock GRBM_GUI_ACTIVE GRBM_COUNT && \
run wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY && \
{ [ -z "${EXTRA_MFMA}" ] || run mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES; } && \
{ [ -z "${EXTRA_L2}" ] || run l2 TCC_HIT_sum TCC_MISS_sum SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD; } && \
echo "pmc ok"
