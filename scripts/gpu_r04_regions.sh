#!/bin/bash
# Round 4: XCD item regions (RT2_ITEM_REGIONS=1: each XCD's workgroups take
# items from their own eighth of the image first) vs one item counter on the
# config B brute-force launch, alternating processes, then the WRITE_SIZE pass
# with regions on (does one XCD per 128-B accumulator line cut the partial-line
# write-backs?).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 0 1 0 1; do
  RT2_ITEM_REGIONS=$r timeout -k 10 200 python scripts/ab_variants.py --config B --variants 263 --rounds 3 > gpurun_out/reg_$r.json 2>&1 || exit 1
  grep median_ms gpurun_out/reg_$r.json | head -1
done
RT2_ITEM_REGIONS=1 timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_reg1 -o run -- python3 bench.py --no-cpu-baseline --no-alt --no-config-c --no-config-e --no-scalar --steps 2 --warmup 1 > gpurun_out/pmc_reg1.log 2>&1 || exit 1
echo done
