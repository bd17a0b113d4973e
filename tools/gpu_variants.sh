#!/bin/bash
# A/B benches of experiment builds (tools/build_variants.py).
#   VARIANTS="ntl nts mb128:march8" bash tools/gpu_variants.sh TAG [bench args]     (name[:stencil-kind])
set -o pipefail
TAG=${1:-variants}; shift
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$OUT/bench_base.log" 2>&1 || exit 2
for VK in $VARIANTS; do
  V=${VK%%:*}; K=${VK#*:}; [ "$K" = "$VK" ] && K=march4
  LIBARG=mp-block-preconditioners_amd/lib/variants/libmpbp_$V.so
  [ "$V" = base ] && LIBARG=
  MPBP_LIB=$LIBARG timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stencil-kind $K "$@" > "$OUT/bench_${V}_$K.log" 2>&1 || exit 3
done
