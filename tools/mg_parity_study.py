"""Where the tolerance-mode ("fast") multigrid apply departs from the exact one (= the oracle's, bit for bit).

    python tools/mg_parity_study.py [--n 256 1024] [--eta 100 1e4]

For each grid and viscosity ratio, one JSON line with relative inf-norm distances to the exact apply of the same
vector:
  fast            the fast apply as the bench runs it (matrix-free level 1, symmetric Gt_F_G half)
  fast_stored_l1  fast, level 1 from the stored Galerkin matrices (kernel options mg_galerkin_mf(_p) = 0)
  fast_full_q13   fast, Gt_F_G from all 13 slots (q13_sym = 0)
  fast_f_only     fast, both of the above (only the fast F rows of level 0 differ)
  ulp_floor       the EXACT apply of the input perturbed by one ulp in every entry: the operator's own forward
                  error -- no fp64 evaluation order can be expected closer to another than this
for the mg:1 / mg:1 apply, the mg:1 / chebyshev:4 and chebyshev:4 / mg:1 splits and the chebyshev:4 headline apply.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[256, 1024])
    ap.add_argument("--eta", type=float, nargs="+", default=[100.0, 1e4])
    args = ap.parse_args()
    import torch
    import mp_block_preconditioners_amd as mp

    def rel(a, b):
        return float((a - b).abs().max() / b.abs().max())

    for n in args.n:
        for eta in args.eta:
            bp = mp.MultiphaseBlockPreconditioner(n, 1.0, eta, 1.0)
            _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
            GtG, GtFG = mp.MultiphaseBlockPreconditioner.commutator_products(F, D, G)
            gen = torch.Generator(device="cuda").manual_seed(n)
            v = torch.randn(5 * n * n, dtype=torch.float64, device="cuda", generator=gen)
            sign = (torch.rand(v.shape, device="cuda", generator=gen, dtype=torch.float64) < 0.5).to(torch.float64)
            v_ulp = v * (1.0 + (2.0 * sign - 1.0) * 2.0 ** -52)   # (float64 throughout: 1 + 2^-52 is a float64 value)
            assert not torch.equal(v_ulp, v)
            line = {"n": n, "eta_n": eta}
            for name, (kf, kp) in {"mg1_mg1": (("mg", 1), ("mg", 1)), "mg1_cheb4": (("mg", 1), ("chebyshev", 4)),
                                   "cheb4_mg1": (("chebyshev", 4), ("mg", 1)),
                                   "cheb4_cheb4": (("chebyshev", 4), ("chebyshev", 4))}.items():
                kw = dict(inner_F=mp.InnerSolver(*kf), inner_P=mp.InnerSolver(*kp))
                ex = mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG, **kw)
                fa = mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG, numerics="fast", **kw)
                ref = ex.apply(v).clone()
                r = {"fast": rel(fa.apply(v), ref)}
                fa.set_kernel_opts(mg_galerkin_mf=0, mg_galerkin_mf_p=0)
                r["fast_stored_l1"] = rel(fa.apply(v), ref)
                fa.set_kernel_opts(q13_sym=0)
                r["fast_f_only"] = rel(fa.apply(v), ref)
                fa.set_kernel_opts(mg_galerkin_mf=2, mg_galerkin_mf_p=1)
                r["fast_full_q13"] = rel(fa.apply(v), ref)
                r["ulp_floor"] = rel(ex.apply(v_ulp), ref)
                line[name] = r
                del ex, fa
                torch.cuda.empty_cache()
            print(json.dumps(line), flush=True)
            del F, D, G, GtG, GtFG, bp
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
