#!/bin/bash
# One GPU session: parity tests, smoke, bench (both layouts), rocprofv3 kernel stats, and a
# 2-rank rehearsal of the row-partitioned bench on the single GPU (gloo).
# usage (on the GPU box, from the repo root): bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu > "$OUT/pytest.log" 2>&1
echo "pytest exit $?" >> "$OUT/pytest.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 10 > "$OUT/bench_sell.log" 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --layout csr --no-cpu-baseline > "$OUT/bench_csr.log" 2>&1 || exit 3
MPBP_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --grid 512 > "$OUT/bench_rows2_gloo.log" 2>&1 || exit 5
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1 || exit 4
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --f-mode assembled --no-cpu-baseline --no-spmv > "$OUT/bench_sell_assembledF.log" 2>&1 || exit 6
# HBM bytes of the F sweeps inside the apply itself (eager launches; the sweeps bench.py times)
for L in stencil sell; do
  FM=auto; [ $L = sell ] && FM=assembled
  for C in FETCH_SIZE WRITE_SIZE; do
    cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/pmc_${L}_$C" -o pmc -- python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-spmv --no-graph --f-mode $FM > "$GRAFT_REPO_ROOT/$OUT/pmc_${L}_$C.log" 2>&1 || exit 7
  done
done
# HBM bytes of the plain A SpMV kernels (tools/spmv_ab.py: CSR per-wave, CSR block, SELL)
for C in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/pmc_spmv_$C" -o pmc -- python "$GRAFT_REPO_ROOT/tools/spmv_ab.py" --reps 10 > "$GRAFT_REPO_ROOT/$OUT/pmc_spmv_$C.log" 2>&1 || exit 11
done
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --pg-mode assembled --no-cpu-baseline --no-spmv > "$OUT/bench_pg_assembled.log" 2>&1 || exit 8
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/sq_stencil" -o pmc -- python "$GRAFT_REPO_ROOT/tools/pmc_sweep.py" --layout stencil > "$GRAFT_REPO_ROOT/$OUT/sq_stencil.log" 2>&1 || exit 9
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/sq2_stencil" -o pmc -- python "$GRAFT_REPO_ROOT/tools/pmc_sweep.py" --layout stencil > "$GRAFT_REPO_ROOT/$OUT/sq2_stencil.log" 2>&1 || exit 10
