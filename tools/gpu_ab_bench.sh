#!/bin/bash
# GPU tests of one file, then SpMV A/B and apply bench A/B of experiment builds.
#   VARIANTS="a b" TESTS=tests/test_gpu_parity.py bash tools/gpu_ab_bench.sh TAG
set -o pipefail
TAG=${1:-ab}
cd "$GRAFT_REPO_ROOT" || exit 9
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/pytest.log" 2>&1 || exit 1
for V in $VARIANTS; do
  MPBP_LIB=mp-block-preconditioners_amd/lib/variants/libmpbp_$V.so timeout -k 10 120 python tools/spmv_ab.py >> "$OUT/spmv_$V.log" 2>&1 || exit 3
  MPBP_LIB=mp-block-preconditioners_amd/lib/variants/libmpbp_$V.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv >> "$OUT/bench_$V.log" 2>&1 || exit 4
done
