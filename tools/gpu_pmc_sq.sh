#!/bin/bash
# SQ counter pass over the F sweep kernels (cells / rows / SELL).  bash tools/gpu_pmc_sq.sh TAG
set -o pipefail
TAG=${1:-pmc}
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for L in stencil sell; do
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/sq_$L" -o pmc -- python "$GRAFT_REPO_ROOT/tools/pmc_sweep.py" --layout $L > "$GRAFT_REPO_ROOT/$OUT/sq_$L.log" 2>&1 || exit 7
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/sq2_$L" -o pmc -- python "$GRAFT_REPO_ROOT/tools/pmc_sweep.py" --layout $L > "$GRAFT_REPO_ROOT/$OUT/sq2_$L.log" 2>&1 || exit 8
done
