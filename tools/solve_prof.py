"""Where FGMRES's time to tolerance goes (bench.py's solve_level case 1024^2, eta_n = 100, mg:1 inner solves).

Runs the solve `--reps` times on one preconditioner (its hipGraph captured once, as bench.py does) and prints one JSON
line per run: wall seconds, iterations, and -- for the first run after torch.cuda.empty_cache() -- what the basis
allocation costs.  Run it under `rocprofv3 --kernel-trace --stats` for the per-kernel split (apply graph, CSR A,
the orthogonalisation's passes, small launches).  --ortho: dcgs2 (the default: rdot2 + dcgs2_update, two basis passes
per iteration), cgs2 (rdot + gs_update twice: four passes), cgs2_fused (the fused update + projection kernel)."""
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
    ap.add_argument("--inner", default="mg:1")
    ap.add_argument("--numerics", default="fast")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ortho", default="dcgs2,cgs2", help="FGMRES orthogonalisations to time, in order")
    args = ap.parse_args()
    import torch
    import mp_block_preconditioners_amd as mp
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import inner_pair
    bp = mp.MultiphaseBlockPreconditioner(args.n, 1.0, args.eta_n, 1.0)
    A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    _, b = mp.manufactured_problem(args.n, xi=1.0, etan=args.eta_n, etas=1.0)
    bd = torch.from_numpy(b).cuda()
    iF, iP = inner_pair(mp, args.inner)
    M = mp.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP, numerics=args.numerics)
    v = torch.randn(M.shape[0], dtype=torch.float64, device="cuda")
    o = torch.empty_like(v)
    g = M.capture(v, o)
    g.replay()
    torch.cuda.synchronize()
    M._fgmres_graph = (v, o, g)
    t0 = time.perf_counter()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    apply_ms = (time.perf_counter() - t0) / 10 * 1e3
    A.matvec(v)   # (the first product builds A's SpMV layout)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        A.matvec(v)
    torch.cuda.synchronize()
    a_ms = (time.perf_counter() - t0) / 10 * 1e3
    for r, mode in ((r, mode) for mode in args.ortho.split(",") for r in range(args.reps)):
        torch.cuda.empty_cache()
        hist = []
        t0 = time.perf_counter()
        x, info = mp.fgmres(A, bd, M=M, tol=1e-8, maxiter=150, residuals=hist, fused_cgs2=mode == "cgs2_fused",
                            ortho="dcgs2" if mode == "dcgs2" else "cgs2")
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        it = len(hist) - 1
        print(json.dumps({"ortho": mode, "rep": r, "seconds": el, "iterations": it, "converged": info == 0, "apply_ms": apply_ms,
                          "A_ms": a_ms, "other_ms_per_iteration": (el * 1e3 - it * (apply_ms + a_ms)) / max(it, 1)}),
              flush=True)
        del x
    t0 = time.perf_counter()
    V = torch.zeros(151, M.shape[0], dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    print(json.dumps({"basis_alloc_zero_ms": (time.perf_counter() - t0) * 1e3, "bytes": V.numel() * 8}), flush=True)


if __name__ == "__main__":
    main()
