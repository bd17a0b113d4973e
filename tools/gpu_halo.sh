#!/bin/bash
# partitioned-path benches on one GPU: RCCL self-exchange, the gloo 2-rank rehearsal.  bash tools/gpu_halo.sh TAG
set -o pipefail
TAG=${1:-halo}
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv --self-halo > "$OUT/bench_selfhalo.log" 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv --no-graph > "$OUT/bench_eager.log" 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-spmv --self-halo > "$OUT/prof.log" 2>&1 || exit 5
MPBP_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --grid 512 > "$OUT/bench_rows2_gloo.log" 2>&1 || exit 6
