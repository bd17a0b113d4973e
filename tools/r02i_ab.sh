#!/bin/bash
# One-off GPU step (round 2): the N > 1 bench path rehearsed with 2 gloo ranks on one GPU at configs[4]'s 2048^2.
cd "$GRAFT_REPO_ROOT" || exit 99
O=gpurun_out/${TAG:-r02aa}; mkdir -p $O
MPBP_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 2 > $O/rows2_gloo_2048.log 2>&1
