#!/bin/bash
# GPU tests + bench over the matrix-free F kernel variants.  bash tools/gpu_sweepkinds.sh TAG
set -o pipefail
TAG=${1:-kinds}
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
[ -n "$NOTEST" ] || timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu > "$OUT/pytest.log" 2>&1
echo "pytest exit $?" >> "$OUT/pytest.log"
for K in ${KINDS:-cells march4 march8}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv --stencil-kind $K > "$OUT/bench_$K.log" 2>&1 || exit 2
done
