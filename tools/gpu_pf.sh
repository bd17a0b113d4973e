#!/bin/bash
# CSR prefetch kernel: parity subset, then SpMV A/B of the SEGS variants.  VARIANTS="segs2 segs8" bash tools/gpu_pf.sh TAG
set -o pipefail
TAG=${1:-pf}
cd "$GRAFT_REPO_ROOT" || exit 9
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "spmv or csr or inner_steps" > "$OUT/pytest.log" 2>&1 || exit 1
VARIANTS="$VARIANTS" bash tools/gpu_spmv_ab.sh "$TAG" || exit 2
