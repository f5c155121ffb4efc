#!/bin/bash
# round 5: resident-kernel neighbours A/B, PMC of the new automatic choice (282), bench + kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/ab_variants.py --config B --variants 282,284,285,286,287 --rounds 3 > gpurun_out/r05b_ab_B.json 2> gpurun_out/r05b_ab_B.err || exit 1
EXTRA_MFMA=1 EXTRA_L2=1 PMC_OUT=gpurun_out/r05b_pmc bash scripts/profile_pmc.sh > gpurun_out/r05b_pmc.log 2>&1 || exit 1
PMC_DIR=gpurun_out/r05b_pmc python3 scripts/parse_pmc.py B > gpurun_out/r05b_pmc_parse.log 2>&1
timeout -k 10 600 python -u bench.py --no-config-c --no-config-e > gpurun_out/r05b_bench.json 2> gpurun_out/r05b_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05b_prof -o run -- python3 bench.py --no-cpu-baseline --no-alt --no-config-c --no-config-e --no-scalar > gpurun_out/r05b_prof.log 2>&1
