#!/bin/bash
# Quick GPU iteration: GPU tests + one bench line (+ the 2-rank gloo rehearsal).  bash tools/gpu_quick.sh TAG [bench args]
set -o pipefail
TAG=${1:-quick}; shift
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu > "$OUT/pytest.log" 2>&1
echo "pytest exit $?" >> "$OUT/pytest.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$OUT/bench.log" 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv --stencil-kind rows > "$OUT/bench_rows.log" 2>&1 || exit 3
MPBP_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --grid 512 > "$OUT/bench_rows2_gloo.log" 2>&1 || exit 5
