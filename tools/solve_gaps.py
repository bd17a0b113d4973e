"""Host-side costs around FGMRES's preconditioner applies (bench.py's time-to-solution case: 1024^2, mg:2 / mg:1).

Prints one JSON line: the host time of one hipGraph launch of the captured apply (g.replay() returning, the GPU idle
before the call), the GPU time of one apply (replays back to back), the CSR A u, and the FGMRES solve's seconds and
iterations -- so the solve's time beyond iterations x (apply + A u) can be set against the launch cost.

    python tools/solve_gaps.py [--n 1024] [--inner mg:2/mg:1] [--eta-n 100]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--eta-n", type=float, default=100.0)
    ap.add_argument("--inner", default="mg:2/mg:1")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import mp_block_preconditioners_amd as mp
    from bench import inner_pair
    bp = mp.MultiphaseBlockPreconditioner(args.n, 1.0, args.eta_n, 1.0)
    A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    _, b = mp.manufactured_problem(args.n, xi=1.0, etan=args.eta_n, etas=1.0)
    bd = torch.from_numpy(b).cuda()
    iF, iP = inner_pair(mp, args.inner)
    M = mp.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP, numerics="fast")
    v = torch.randn(M.shape[0], dtype=torch.float64, device="cuda")
    o = torch.empty_like(v)
    g = M.capture(v, o)
    g.replay()
    torch.cuda.synchronize()
    M._fgmres_graph = (v, o, g)
    calls = []
    for _ in range(10):   # the host cost of one launch, the queue empty
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        calls.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    apply_ms = (time.perf_counter() - t0) / 10 * 1e3
    A.matvec(v)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        A.matvec(v)
    torch.cuda.synchronize()
    a_ms = (time.perf_counter() - t0) / 10 * 1e3
    solves = []
    for _ in range(args.reps):
        hist = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mp.fgmres(A, bd, M=M, tol=1e-8, maxiter=150, residuals=hist)
        torch.cuda.synchronize()
        solves.append({"seconds": round(time.perf_counter() - t0, 5), "iterations": len(hist) - 1})
    it = solves[-1]["iterations"]
    print(json.dumps({"n": args.n, "eta_n": args.eta_n, "inner": args.inner,
                      "graph_launch_host_ms": [round(c * 1e3, 3) for c in calls], "apply_ms": round(apply_ms, 4),
                      "A_ms": round(a_ms, 4), "solves": solves,
                      "beyond_applies_ms_per_iteration": round((solves[-1]["seconds"] * 1e3 - it * (apply_ms + a_ms))
                                                               / max(it, 1), 4)}), flush=True)


if __name__ == "__main__":
    main()
