#!/bin/bash
# One-off GPU step (round 2): the auto rows-per-workgroup default at 256^2, 1024^2 and 2048^2 (one GPU).
cd "$GRAFT_REPO_ROOT" || exit 99
O=gpurun_out/${TAG:-r02af}; mkdir -p $O
B="timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-spmv --no-solve"
for G in 256 1024 2048; do $B --grid $G > $O/g${G}_auto.log 2>&1 || exit 1; done
