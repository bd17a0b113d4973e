#!/bin/bash
# GPU tests + benches (matrix-free D/G/Gt_G on / off) + a kernel-trace profile.  bash tools/gpu_pg.sh TAG
set -o pipefail
TAG=${1:-pg}
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu > "$OUT/pytest.log" 2>&1
  rc=$?
  echo "pytest exit $rc" >> "$OUT/pytest.log"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench.log" 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv --pg-mode assembled > "$OUT/bench_pg_assembled.log" 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-spmv --no-graph > "$OUT/prof.log" 2>&1 || exit 5
MPBP_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --grid 512 > "$OUT/bench_rows2_gloo.log" 2>&1 || exit 6
