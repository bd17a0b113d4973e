"""Solve-level study: FGMRES (tol 1e-8, maxiter 150, x0 = 0, solve.py:285) on the reference's manufactured problem
(solve.py:52-80) with the approximate Schur preconditioner and mixed inner solves, plus the graph-replayed apply rate
of each preconditioner and its level sizes (multigrid).  One JSON line per run.

    python tools/solve_study.py [--n 256 1024] [--eta-n 100 1e4] [--combos cheb4/mg1 mg1/mg1 ...]

Combos are F/P inner solvers: chebN = N Chebyshev-Jacobi sweeps, jacN = N Jacobi sweeps, mgN = N V-cycles.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def inner(mp, spec, **mgkw):
    for pre, kind in (("cheb", "chebyshev"), ("jac", "jacobi"), ("mg", "mg")):
        if spec.startswith(pre):
            return mp.InnerSolver(kind, int(spec[len(pre):]), **(mgkw if kind == "mg" else {}))
    raise ValueError(spec)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[256, 1024])
    ap.add_argument("--eta-n", type=float, nargs="+", default=[100.0, 1e4])
    ap.add_argument("--combos", nargs="+", default=["cheb4/cheb4", "mg1/mg1", "cheb4/mg1", "cheb8/mg1", "mg1/cheb4",
                                                      "mg2/mg1"])
    ap.add_argument("--pre", type=int, default=2)
    ap.add_argument("--post", type=int, default=2)
    ap.add_argument("--coarsest", type=int, default=16)
    ap.add_argument("--smooth-ratio", type=float, default=4.0)
    ap.add_argument("--tol", type=float, default=1e-8)
    ap.add_argument("--maxiter", type=int, default=150)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tag", default="")
    ap.add_argument("--solves", type=int, default=1, help="solves per combo (the last one reported; all in solve_times)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import mp_block_preconditioners_amd as mp
    mgkw = dict(pre=args.pre, post=args.post, coarsest=args.coarsest, smooth_ratio=args.smooth_ratio)
    for n in args.n:
        for eta_n in args.eta_n:
            bp = mp.MultiphaseBlockPreconditioner(n, 1.0, eta_n, 1.0)
            A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
            u, b = mp.manufactured_problem(n, xi=1.0, etan=eta_n, etas=1.0)
            bd = torch.from_numpy(b).cuda()
            nb = float(torch.linalg.vector_norm(bd))
            for combo in args.combos:
                fs, ps = combo.split("/")
                t0 = time.perf_counter()
                M = mp.ApproxSchurPreconditioner(F, D, G, inner_F=inner(mp, fs, **mgkw), inner_P=inner(mp, ps, **mgkw))
                torch.cuda.synchronize()
                setup = time.perf_counter() - t0
                # apply rate: graph replay of one apply on a random vector
                v = torch.randn(M.shape[0], dtype=torch.float64, device="cuda")
                out = torch.empty_like(v)
                g = M.capture(v, out)
                g.replay()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.reps):
                    g.replay()
                torch.cuda.synchronize()
                apply_ms = (time.perf_counter() - t0) / args.reps * 1e3
                del g
                times = []
                for _ in range(args.solves):   # later solves reuse the captured apply (fgmres keeps it on M)
                    hist = []
                    t0 = time.perf_counter()
                    x, info = mp.fgmres(A, bd, M=M, tol=args.tol, maxiter=args.maxiter, residuals=hist)
                    torch.cuda.synchronize()
                    times.append(time.perf_counter() - t0)
                el = times[-1]
                res = float(torch.linalg.vector_norm(bd - A.matvec(x))) / nb
                err = float(np.max(np.abs(x.cpu().numpy()[: 4 * n * n] - u[: 4 * n * n])))
                levels = {k: (m.sizes if m is not None else None) for k, m in (("F", M.mg_F), ("P", M.mg_P))}
                nnz = {k: ([op.nnz for op in m.ops] if m is not None else None) for k, m in (("F", M.mg_F), ("P", M.mg_P))}
                print(json.dumps({"tag": args.tag, "coarsest": args.coarsest, "pre": args.pre, "post": args.post,
                                  "smooth_ratio": args.smooth_ratio, "n": n, "eta_n": eta_n, "combo": combo, "iterations": len(hist) - 1,
                                  "converged": info == 0, "solve_s": el, "solve_times": times, "setup_s": setup, "apply_ms": apply_ms,
                                  "ms_per_iteration": el / max(1, len(hist) - 1) * 1e3, "true_rel_residual": res,
                                  "velocity_max_error": err, "mg_levels": levels, "mg_nnz": nnz,
                                  "residuals": [float(r) for r in hist[:: max(1, len(hist) // 10)]]}), flush=True)
                del M, x, v, out
                torch.cuda.empty_cache()
            del A, F, D, G, bp
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
