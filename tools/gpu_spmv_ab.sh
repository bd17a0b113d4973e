#!/bin/bash
# A/B of CSR SpMV experiment builds: VARIANTS="tg cap640" bash tools/gpu_spmv_ab.sh TAG
set -o pipefail
TAG=${1:-spmv_ab}
cd "$GRAFT_REPO_ROOT" || exit 9
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 120 python tools/spmv_ab.py > "$OUT/base.log" 2>&1 || exit 2
for V in $VARIANTS; do
  MPBP_LIB=mp-block-preconditioners_amd/lib/variants/libmpbp_$V.so timeout -k 10 120 python tools/spmv_ab.py > "$OUT/$V.log" 2>&1 || exit 3
done
