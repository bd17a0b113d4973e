#!/bin/bash
# stencil / fusion GPU tests, then benches with and without the two-sweep fusion + kernel trace.  bash tools/gpu_fuse.sh TAG
set -o pipefail
TAG=${1:-fuse}
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py tests/test_gpu_pg_stencil.py -x -q --timeout 300 --timeout-method thread -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 4
for R in 8 4 16 0; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv --sweep-fusion $R > "$OUT/bench_f$R.log" 2>&1 || exit 2
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-spmv --no-graph > "$OUT/prof.log" 2>&1 || exit 5
