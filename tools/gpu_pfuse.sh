#!/bin/bash
# bench over the one-pass Gt_G solve's rows per workgroup.  bash tools/gpu_pfuse.sh TAG
set -o pipefail
TAG=${1:-pfuse}
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for R in ${ROWS:-0 2 4 8 16}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv --p-fusion $R > "$OUT/bench_p$R.log" 2>&1 || exit 2
done
