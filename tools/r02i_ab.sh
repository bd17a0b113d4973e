#!/bin/bash
# One-off GPU step list (round 2): parity + MG tests, then the solve study at 1024^2 with the new orthogonalisation.
cd "$GRAFT_REPO_ROOT" || exit 99
O=gpurun_out/${TAG:-r02v}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mg.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/solve_study.py --n 256 1024 --eta-n 100 1e4 --combos cheb4/cheb4 mg1/mg1 mg2/mg1 --tag gs >> $O/study.log 2>&1
