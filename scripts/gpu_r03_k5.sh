#!/bin/bash
# Round 3, session 2: the 5-product form (variants 227-230) against variant 200:
# config B whole image (bit-identical images asserted), config C and E samples,
# rank slabs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export RT2_LIB=exp
timeout -k 10 300 python scripts/ab_variants.py --variants "${AB_B:-200,227,230,210,229}" --rounds 3 > gpurun_out/k5_ab_B.log 2>&1 || { echo "ab B failed"; exit 1; }
timeout -k 10 300 python scripts/ab_variants.py --config C --width 480 --height 270 --frames 2 --variants "${AB_C:-200,227,230}" --rounds 2 > gpurun_out/k5_ab_C.log 2>&1 || { echo "ab C failed"; exit 1; }
timeout -k 10 300 python scripts/shard_probe.py --variants "${SHARD:-0,227,228}" > gpurun_out/k5_shard.log 2>&1 || { echo "shard failed"; exit 1; }
timeout -k 10 300 python scripts/ab_variants.py --config E --width 480 --height 270 --variants "${AB_E:-200,227}" --rounds 1 > gpurun_out/k5_ab_E.log 2>&1 || { echo "ab E failed"; exit 1; }
echo "all ok"
