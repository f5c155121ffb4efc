#!/bin/bash
# round 5: the slab kernel's cooperative-drain threshold under fair-share priority (298: 4 live rays;
# 306: 8; 307: 0; 308: 16): every rank's slab, config B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RT2_LIB=exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 120 --timeout-method thread -k "v306 or v307 or v308" > gpurun_out/r05u_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/shard_probe.py --config B --variants 298,306,307,308 --ns 2,4,8 --reps 2 > gpurun_out/r05u_shard_B.jsonl 2> gpurun_out/r05u_shard_B.err
