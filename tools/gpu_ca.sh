#!/bin/bash
# CA schedule check: distributed GPU tests, single-GPU parity subset, benches (single, self-halo CA / per-sweep,
# gloo 2-rank rehearsal).   bash tools/gpu_ca.sh TAG
set -o pipefail
TAG=${1:-ca}
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_dist.log" 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py tests/test_gpu_pg_stencil.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_par.log" 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv > "$OUT/bench_single.log" 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv --self-halo > "$OUT/bench_selfhalo_ca.log" 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv --self-halo --no-ca > "$OUT/bench_selfhalo_sweep.log" 2>&1 || exit 5
MPBP_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --grid 512 > "$OUT/bench_rows2_gloo.log" 2>&1 || exit 6
