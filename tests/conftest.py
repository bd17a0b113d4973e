import glob
import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def golden_files():
    return sorted(glob.glob(os.path.join(GOLDEN_DIR, "golden_n*.npz")))


def load_golden(path):
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


def golden_csr(g, name):
    return sp.csr_matrix((g[name + "_data"], g[name + "_indices"], g[name + "_indptr"]),
                         shape=tuple(int(s) for s in g[name + "_shape"]))


def golden_params(g):
    n, xi, eta_n, eta_s, c, d, d_p, d_div = g["params"]
    return dict(n=int(n), xi=float(xi), eta_n=float(eta_n), eta_s=float(eta_s), c=float(c),
                d_u=float(d), d_p=float(d_p), d_div=float(d_div))


def golden_tables(g):
    """The thn tables a fixture was generated with: None (the reference's variable thn, preconditioner.py:9-11)
    or constant tables for the constant-thn cases (BASELINE configs[0], solve.py:60-68)."""
    if "theta_const" not in g:
        return None
    n = golden_params(g)["n"]
    t = np.full(n * n, float(g["theta_const"]))
    return t, t.copy(), t.copy()


def rel_inf(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.max(np.abs(b)), 1e-300)
    return float(np.max(np.abs(a - b)) / scale)


@pytest.fixture(scope="session")
def oracle_built():
    from oracle import csr_oracle
    csr_oracle.build()
    return True
