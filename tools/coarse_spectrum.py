"""Singular values of the coarsest Galerkin operators (oracle hierarchy, coarsest 16^2) for F and Gt_G: the evidence
behind mg.COARSE_RCOND (where the pseudo-inverse's null-space cut sits).

    PYTHONPATH=. python tools/coarse_spectrum.py 256 1024 [--eta 100 1e4]
"""
import argparse
import time

import numpy as np

from oracle import mg_oracle as mo
from oracle.stokes_oracle import StokesSystem


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", type=int, nargs="+")
    ap.add_argument("--eta", type=float, nargs="+", default=[100.0, 1e4])
    args = ap.parse_args()
    for n in args.n:
        for eta in args.eta:
            t = time.time()
            s = StokesSystem(n, 1.0, eta, 1.0, 1.0, -1.0, products=True)
            for name, M, f in (("F", s.F, mo.FIELDS_VELOCITY), ("GtG", s.GtG, mo.FIELDS_PRESSURE)):
                ops, _, _ = mo.hierarchy(M, n, f, coarsest=16)
                sv = np.linalg.svd(ops[-1][0].toarray(), compute_uv=False)
                print(f"n={n} eta={eta:g} {name} {ops[-1][0].shape}: sigma_max {sv[0]:.3e}, five smallest / sigma_max "
                      + " ".join(f"{v:.2e}" for v in sv[-5:][::-1] / sv[0]) + f"  ({time.time() - t:.0f} s)", flush=True)


if __name__ == "__main__":
    main()
