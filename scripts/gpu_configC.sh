#!/bin/bash
# Config C (100k triangles), brute force: GPU parity of the large-scene paths,
# one full bench step (1920x1080, 64 rays x 4 frames), then HBM-traffic PMC
# passes on a reduced-spp render of the same scene (the traffic per test is
# what matters).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "tiled or auto_variant or brute_variants" > gpurun_out/t.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 400 python -u bench.py --config C --traversal brute --steps 1 --warmup 0 --no-alt --no-cpu-baseline > gpurun_out/bench_C_brute.log 2>&1 || { echo "bench C failed"; exit 1; }
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcp_C_$c" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/ab_variants.py" --config C --rays 2 --variants ${VARIANT:-0} --rounds 1 > "$GRAFT_REPO_ROOT/gpurun_out/pmcp_C_$c.log" 2>&1 || { echo "pmc $c failed"; exit 1; }
done
echo "all ok"
