#!/bin/bash
# One-off GPU step (round 2): Gram-Schmidt kernel tests, then a kernel trace of the 1024^2 FGMRES solves.
cd "$GRAFT_REPO_ROOT" || exit 99
O=gpurun_out/${TAG:-r02x}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mg.py -x -q --timeout 240 --timeout-method thread -m gpu -k "gram or fgmres" > $O/pytest.log 2>&1 || exit 1
(cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o run -- \
   python "$GRAFT_REPO_ROOT/tools/solve_study.py" --n 1024 --eta-n 100 --combos mg1/mg1 cheb4/cheb4 --tag prof) > $O/prof.log 2>&1
