#!/bin/bash
# One-off GPU step list (round 2): multigrid tests, then solve-study A/B runs at 1024^2.
cd "$GRAFT_REPO_ROOT" || exit 99
O=gpurun_out/${TAG:-r02j}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || exit 1
S="timeout -k 10 200 python -u tools/solve_study.py --n 1024 --eta-n 100 1e4 --combos mg1/mg1 mg2/mg1"
$S --tag c16 >> $O/study.log 2>&1 && $S --coarsest 8 --tag c8 >> $O/study.log 2>&1
