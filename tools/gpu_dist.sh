#!/bin/bash
# distributed-path GPU tests + self-exchange benches (in order / overlap) + kernel trace.  bash tools/gpu_dist.sh TAG
set -o pipefail
TAG=${1:-dist}
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/pytest.log"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv --self-halo > "$OUT/bench_inorder.log" 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv --self-halo --halo-overlap > "$OUT/bench_overlap.log" 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-spmv --self-halo > "$OUT/prof.log" 2>&1 || exit 5
