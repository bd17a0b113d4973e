#!/bin/bash
# One-off GPU step (round 2): A/B of the CSR SpMV LDS swizzle (tools/spmv_ab.py per build, interleaved).
cd "$GRAFT_REPO_ROOT" || exit 99
O=gpurun_out/${TAG:-r02z}; mkdir -p $O
for V in base swz base swz base swz; do
  L=mp-block-preconditioners_amd/lib/variants/libmpbp_$V.so; [ $V = base ] && L=
  MPBP_LIB=$L timeout -k 10 120 python tools/spmv_ab.py >> $O/spmv_$V.log 2>&1 || exit 1
done
