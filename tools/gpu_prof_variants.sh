#!/bin/bash
# kernel traces of the default bench apply for experiment builds.  VARIANTS="a b" bash tools/gpu_prof_variants.sh TAG
set -o pipefail
TAG=${1:-profvar}
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for V in base $VARIANTS; do
  LIBARG=mp-block-preconditioners_amd/lib/variants/libmpbp_$V.so
  [ "$V" = base ] && LIBARG=
  MPBP_LIB=$LIBARG timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_$V" -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-spmv > "$OUT/prof_$V.log" 2>&1 || exit 2
done
