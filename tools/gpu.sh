#!/bin/bash
# The one GPU-box launcher: runs named steps in order, each under its own time limit, logs under
# gpurun_out/TAG/, and stops at the first step that fails (a test failure, a GPU fault, a time limit).
#
#   gpurun --timeout 1200 -- bash tools/gpu.sh TAG tests smoke bench ...
#
# Steps:
#   tests        pytest -m gpu (all GPU parity tests)          smoke     __graft_entry__.smoke()
#   tests:F1,F2  pytest -m gpu of the named test files / node ids only
#   bench        bench.py, N = 1 (the driver's command)        bench_csr bench.py --layout csr
#   bench:ARGS   bench.py ARGS ('+' for spaces; MPBP_BENCH_BACKEND etc. from the environment), appended to bench_args.log
#   rows2_gloo   bench.py --gpus 2 --grid 512 over gloo on one GPU (the N > 1 path; launcher inside bench.py)
#   gloo:N       bench.py --gpus N (configs[4]'s 2048^2) over gloo on one GPU: the N > 1 line's sections rehearsed
#   selfhalo     bench.py --self-halo (partitioned apply over the RCCL self-exchange)
#   probe        tools/capture_probe.py 256 1024 (hipGraph capture of the partitioned apply); probe:N1,N2 sizes
#   prof         rocprofv3 --kernel-trace --stats of bench.py
#   profmg       the same with the headline apply's inner solves one multigrid V-cycle each (mg:1 / mg:1)
#   profsolve    the same over tools/solve_prof.py (FGMRES to 1e-8 on 1024^2, mg:1 inner solves; args in $SOLVE_ARGS)
#   pmc          FETCH_SIZE / WRITE_SIZE passes: the apply's F sweeps and the A SpMV
#   sq           SQ counter passes over the F sweep (tools/pmc_sweep.py) and the CSR SpMV (tools/spmv_ab.py)
#   spmvattr     FETCH_SIZE / WRITE_SIZE of the A SpMV against the same matrix with its x gathers in a 32 KB window
#   sqmg         the same over the multigrid apply (mg:1 / mg:1 inner solves; extra bench args in $SQMG_ARGS)
#   sqapply      SQ counter passes over bench.py's eager apply (every kernel of the apply; tools/pmc_table.py)
#   setup:ARGS   tools/setup_timing.py ARGS ('+' for spaces): the partitioned preconditioner's setup over gloo ranks on one GPU
#   py:FILE      python FILE (any experiment script), 300 s
#   ab:V1,V2,..  A/B of experiment builds (tools/build_variants.py): bench.py per variant (V or V@ARGS, '+' for
#                spaces; variant "base" = the product library); extra bench args for all in $BENCH_ARGS
#   spmv:V1,..   tools/spmv_ab.py (the A SpMV kernels) per variant
set -o pipefail
TAG=${1:-run}
shift
cd "$GRAFT_REPO_ROOT" || exit 99
export TMPDIR=/tmp
ROOTD=$GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p "$OUT"

prof() {   # prof NAME TIMEOUT ARGS... : rocprofv3 run from /tmp with the program right after --
  local name=$1 t=$2
  shift 2
  (cd /tmp && timeout -s KILL "$t" rocprofv3 "$@") > "$ROOTD/$OUT/$name.log" 2>&1
}

step() {
  local s=$1
  echo "== $s $(date +%T)"
  case $s in
    tests) timeout -k 10 1000 python -u -m pytest tests/ -x -v --timeout 240 --timeout-method thread -m gpu \
             > "$OUT/pytest.log" 2>&1 ;;
    tests:*) timeout -k 10 900 python -u -m pytest $(echo "${s#tests:}" | tr , ' ') -x -q --timeout 240 \
               --timeout-method thread -m gpu > "$OUT/pytest_part.log" 2>&1 ;;
    smoke) timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench) timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 ;;
    bench:*) local A=$(echo "${s#bench:}" | tr + ' ')   # bench.py with extra arguments ('+' for spaces)
          timeout -k 10 400 python bench.py $A >> "$OUT/bench_args.log" 2>&1 ;;
    bench_csr) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --layout csr --no-cpu-baseline \
                 > "$OUT/bench_csr.log" 2>&1 ;;
    rows2_gloo) MPBP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --grid 512 \
                  > "$OUT/rows2_gloo.log" 2>&1 ;;
    gloo:*) MPBP_BENCH_BACKEND=gloo timeout -k 10 900 python bench.py --gpus ${s#gloo:} --steps 5 --warmup 2 \
              > "$OUT/gloo_${s#gloo:}.log" 2>&1 ;;
    selfhalo) timeout -k 10 300 python bench.py --self-halo --steps 20 --warmup 5 --no-cpu-baseline --no-spmv \
                > "$OUT/selfhalo.log" 2>&1 ;;
    probe) timeout -k 10 120 python -u tools/capture_probe.py 256 1024 > "$OUT/probe.log" 2>&1 ;;
    probe:*) timeout -k 10 120 python -u tools/capture_probe.py $(echo "${s#probe:}" | tr , ' ') \
               > "$OUT/probe_${s#probe:}_${MPBP_HALO_CAPTURED_DESTROY:-leak}.log" 2>&1 ;;
    prof) prof prof 300 --kernel-trace --stats --output-format csv -d "$ROOTD/$OUT/prof" -o run -- \
            python "$ROOTD/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-solve $BENCH_ARGS &&
          python tools/prof_summary.py "$OUT/prof/run_kernel_trace.csv" > "$OUT/prof_summary.md" 2>&1 ;;
    profmg) prof prof_mg 300 --kernel-trace --stats --output-format csv -d "$ROOTD/$OUT/prof_mg" -o run -- \
              python "$ROOTD/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-solve --no-mg --no-spmv \
              --inner-f mg:1 --inner-p mg:1 &&
            python tools/prof_summary.py "$OUT/prof_mg/run_kernel_trace.csv" > "$OUT/prof_mg_summary.md" 2>&1 ;;
    profsolve) prof prof_solve 300 --kernel-trace --stats --output-format csv -d "$ROOTD/$OUT/prof_solve" -o run -- \
                 python "$ROOTD/tools/solve_prof.py" --reps 2 $SOLVE_ARGS &&
               python tools/prof_summary.py "$OUT/prof_solve/run_kernel_trace.csv" > "$OUT/prof_solve_summary.md" 2>&1 ;;
    pmc) for C in FETCH_SIZE WRITE_SIZE; do
           prof "pmc_apply_$C" 150 --pmc $C --output-format csv -d "$ROOTD/$OUT/pmc_apply_$C" -o pmc -- \
             python "$ROOTD/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-spmv --no-graph --no-solve || return 1
           prof "pmc_spmv_$C" 120 --pmc $C --output-format csv -d "$ROOTD/$OUT/pmc_spmv_$C" -o pmc -- \
             python "$ROOTD/tools/spmv_ab.py" --reps 10 || return 1
         done ;;
    spmvattr) for C in FETCH_SIZE WRITE_SIZE; do
           prof "spmvattr_$C" 150 --pmc $C --output-format csv -d "$ROOTD/$OUT/spmvattr/pmc_$C" -o pmc -- \
             python "$ROOTD/tools/spmv_attr.py" --reps 10 || return 1
         done && python tools/spmv_attr.py --reduce "$OUT/spmvattr" > "$OUT/spmv_attr.json" 2>&1 &&
         timeout -k 10 120 python tools/spmv_attr.py --reps 50 >> "$OUT/spmv_attr.json" 2>&1 ;;
    sq) for W in "pmc_sweep.py --layout stencil" "spmv_ab.py --reps 10"; do
          local tag=${W%%.py*}
          prof "sq1_$tag" 120 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d "$ROOTD/$OUT/sq1_$tag" \
            -o pmc -- python "$ROOTD/tools/"$W || return 1
          prof "sq2_$tag" 120 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS \
            SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT --output-format csv \
            -d "$ROOTD/$OUT/sq2_$tag" -o pmc -- python "$ROOTD/tools/"$W || return 1
        done ;;
    ab:*) local V   # VARIANT[@ARGS] (ARGS with '+' for spaces), e.g. ab:base,mb128@--march-rows+8
          for V in $(echo "${s#ab:}" | tr , ' '); do
            local N=${V%%@*} A=""
            [ "$N" != "$V" ] && A=$(echo "${V#*@}" | tr + ' ')
            local L=mp-block-preconditioners_amd/lib/variants/libmpbp_$N.so
            [ "$N" = base ] && L=
            MPBP_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv $A \
              $BENCH_ARGS >> "$OUT/ab_bench_$N$(echo "$A" | tr -d ' -').log" 2>&1 || return 1
          done ;;
    spmv:*) local V
          for V in $(echo "${s#spmv:}" | tr , ' '); do
            local L=mp-block-preconditioners_amd/lib/variants/libmpbp_$V.so
            [ "$V" = base ] && L=
            MPBP_LIB=$L timeout -k 10 120 python tools/spmv_ab.py >> "$OUT/spmv_$V.log" 2>&1 || return 1
          done ;;
    sqapply|sqmg) local B="$ROOTD/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-spmv --no-graph"
          [ "$s" = sqmg ] && B="$B --no-mg --no-solve --inner-f mg:1 --inner-p mg:1 $SQMG_ARGS"
          prof sq1_apply 150 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d "$ROOTD/$OUT/sq1_apply" \
            -o pmc -- python $B || return 1
          prof sq2_apply 150 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS \
            SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT --output-format csv \
            -d "$ROOTD/$OUT/sq2_apply" -o pmc -- python $B || return 1
          # reduce on the box (the raw per-dispatch CSVs of a whole bench run exceed gpurun's 64 MiB copy-back)
          mkdir -p "$OUT/sqraw" && mv "$OUT"/sq1_apply "$OUT"/sq2_apply "$OUT/sqraw/" &&
            python tools/pmc_table.py "$OUT/sqraw" --json "$OUT/sq_$s.json" > "$OUT/sq_$s.txt" &&
            rm -rf "$OUT/sqraw" ;;
    setup:*) timeout -k 10 600 python -u tools/setup_timing.py $(echo "${s#setup:}" | tr + ' ') >> "$OUT/setup_timing.log" 2>&1 ;;
    py:*) timeout -k 10 300 python -u "${s#py:}" > "$OUT/$(basename "${s#py:}" .py).log" 2>&1 ;;
    *) echo "unknown step $s"; return 98 ;;
  esac
}

i=0
for s in "$@"; do
  i=$((i + 1))
  step "$s"
  rc=$?
  echo "== $s exit $rc"
  if [ $rc -ne 0 ]; then
    echo "step $s failed ($rc): stopping" | tee -a "$OUT/steps.log"
    exit $i
  fi
  echo "$s ok" >> "$OUT/steps.log"
done
