"""Generate the golden fixtures in tests/golden/ from the reference itself.

Run in the build container (the reference is NOT available on the GPU box):

    python tests/golden/make_golden.py /root/reference

The reference's ``preconditioner.py`` and ``utils.py`` need only numpy/scipy/pandas and are
executed from their source text (no cached bytecode is loaded).  ``solve.py`` imports
petsc4py / slepc4py / ilupp / pyamg / sympy, which are absent, so the two pieces of it the
fixtures need are restated below with their file:line:

* ``Jacobi(A, b, N, x)``                                  solve.py:149-159
* the approximate-commutator products Gt_G, Gt_F_G        solve.py:246-249
* the body of ``approx_schur_op(v)``                       solve.py:257-277, with the two ILU
  factorizations (ilupp, absent) replaced by (a) exact inverses and (b) N Jacobi sweeps.

Outputs: ``golden_n{n}_{tag}.npz`` -- dense reference matrices stored as CSR of their nonzeros
plus input/output vectors.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
PI = np.pi

CASES = [
    # tag, n, xi, eta_n, eta_s, c, d
    ("unit", 2, 1.0, 1.0, 1.0, 1.0, -1.0),
    ("unit", 3, 1.0, 1.0, 1.0, 1.0, -1.0),
    ("unit", 4, 1.0, 1.0, 1.0, 1.0, -1.0),
    ("unit", 5, 1.0, 1.0, 1.0, 1.0, -1.0),
    ("unit", 8, 1.0, 1.0, 1.0, 1.0, -1.0),
    ("visc", 8, 1.0, 100.0, 1.0, 1.0, -1.0),      # solve.py:291-297 parameters
    ("visc", 16, 1.0, 100.0, 1.0, 1.0, -1.0),
    ("stiff", 8, 2.5, 1.0e4, 1.0, 1.0, -1.0),      # BASELINE configs[3]: eta_n/eta_s = 1e4
]
BIG = [("visc", 32, 1.0, 100.0, 1.0, 1.0, -1.0)]   # A, u_vec, b_vec, A @ u_vec only
# BASELINE configs[0]: the reference's "Fixed Thn = 0.75" manufactured problem (solve.py:60-68): the
# reference's own thn (preconditioner.py:9-11) replaced by the constant 0.75 in the executed module.
CONST = [("const75", 8, 1.0, 1.0, 1.0, 1.0, -1.0, False), ("const75", 32, 1.0, 1.0, 1.0, 1.0, -1.0, True)]
THETA_CONST = 0.75


def load_reference(ref_dir):
    sys.dont_write_bytecode = True
    mods = {}
    for name in ("preconditioner", "utils"):
        path = os.path.join(ref_dir, name + ".py")
        with open(path) as f:
            src = f.read()
        mod = types.ModuleType(name)
        mod.__file__ = path
        sys.modules[name] = mod
        exec(compile(src, path, "exec"), mod.__dict__)
        mods[name] = mod
    return mods["preconditioner"], mods["utils"]


def jacobi(A, b, N, x):
    """solve.py:149-159: x = (b - R x) / D, N times."""
    D = np.diag(A)
    R = A - np.diagflat(D)
    for _ in range(N):
        x = (b - np.dot(R, x)) / D
    return x


def manufactured(n, c, d, xi, etan, etas, utils):
    """u_vec, b_vec of the variable-thn manufactured problem (solve.py:52-80)."""
    nu = 1.0
    u_n_x = lambda y, x: np.sin(2 * PI * x) * np.cos(2 * PI * y)
    u_n_y = lambda y, x: np.cos(2 * PI * x) * np.sin(2 * PI * y)
    u_s_x = lambda y, x: -np.sin(2 * PI * x) * np.cos(2 * PI * y)
    u_s_y = lambda y, x: -np.cos(2 * PI * x) * np.sin(2 * PI * y)
    p_f = lambda y, x: 0.0
    S2 = lambda a: np.sin(2 * PI * a)
    C2 = lambda a: np.cos(2 * PI * a)
    b_n_x = lambda y, x: (C2(y) * S2(x) * (4 * c * nu - 4 * d * (8 * etan * nu * PI * PI + xi) + 2 * nu * (c - 16 * d * etan * PI * PI) * S2(x) * S2(y) + d * xi * S2(x) * S2(x) * S2(y) * S2(y))) / (8 * nu)
    b_n_y = lambda y, x: (C2(x) * S2(y) * (4 * c * nu - 4 * d * (8 * etan * nu * PI * PI + xi) + 2 * nu * (c - 16 * d * etan * PI * PI) * S2(x) * S2(y) + d * xi * S2(x) * S2(x) * S2(y) * S2(y))) / (8 * nu)
    b_s_x = lambda y, x: (C2(y) * S2(x) * (-4 * c * nu + 4 * d * (8 * etas * nu * PI * PI + xi) + 2 * nu * (c - 16 * d * etas * PI * PI) * S2(x) * S2(y) - d * xi * S2(x) * S2(x) * S2(y) * S2(y))) / (8 * nu)
    b_s_y = lambda y, x: (C2(x) * S2(y) * (-4 * c * nu + 4 * d * (8 * etas * nu * PI * PI + xi) + 2 * nu * (c - 16 * d * etas * PI * PI) * S2(x) * S2(y) - d * xi * S2(x) * S2(x) * S2(y) * S2(y))) / (8 * nu)
    b_p = lambda y, x: -PI * np.sin(4 * PI * x) * np.sin(4 * PI * y)
    return utils.fill_sol_and_RHS_vecs(n, u_n_x, u_n_y, u_s_x, u_s_y, p_f, b_n_x, b_n_y, b_s_x, b_s_y, b_p)


def manufactured_const75(n, c, d, xi, etan, etas, utils):
    """u_vec, b_vec of the constant-thn (0.75) manufactured problem: the RHS expressions the reference keeps
    commented out at solve.py:62-68 (same solution components, solve.py:52-58)."""
    nu = 1.0
    u_n_x = lambda y, x: np.sin(2 * PI * x) * np.cos(2 * PI * y)
    u_n_y = lambda y, x: np.cos(2 * PI * x) * np.sin(2 * PI * y)
    u_s_x = lambda y, x: -np.sin(2 * PI * x) * np.cos(2 * PI * y)
    u_s_y = lambda y, x: -np.cos(2 * PI * x) * np.sin(2 * PI * y)
    p_f = lambda y, x: 0.0
    b_n_x = lambda y, x: (3 * (2 * c * nu - d * (16 * etan * nu * PI * PI + xi)) * np.cos(2 * PI * y) * np.sin(2 * PI * x)) / (8 * nu)
    b_n_y = lambda y, x: (3 * (2 * c * nu - d * (16 * etan * nu * PI * PI + xi)) * np.cos(2 * PI * x) * np.sin(2 * PI * y)) / (8 * nu)
    b_s_x = lambda y, x: ((-2 * c * nu + 16 * d * etas * nu * PI * PI + 3 * d * xi) * np.cos(2 * PI * y) * np.sin(2 * PI * x)) / (8 * nu)
    b_s_y = lambda y, x: ((-2 * c * nu + 16 * d * etas * nu * PI * PI + 3 * d * xi) * np.cos(2 * PI * x) * np.sin(2 * PI * y)) / (8 * nu)
    b_p = lambda y, x: -2 * PI * np.cos(2 * PI * x) * np.cos(2 * PI * y)
    return utils.fill_sol_and_RHS_vecs(n, u_n_x, u_n_y, u_s_x, u_s_y, p_f, b_n_x, b_n_y, b_s_x, b_s_y, b_p)


def csr_fields(prefix, M):
    M = sp.csr_matrix(M)
    M.sort_indices()
    return {prefix + "_data": M.data, prefix + "_indices": M.indices.astype(np.int32),
            prefix + "_indptr": M.indptr.astype(np.int32), prefix + "_shape": np.array(M.shape)}


def approx_schur(F, D, G, v, finv, gtg_inv, Gt_F_G):
    """Body of approx_schur_op (solve.py:257-277) with pluggable inner inverses."""
    Finv_v = finv(v[:F.shape[1]])
    rhs_interim = np.matmul(D, Finv_v) + v[F.shape[1]:]
    x_a = gtg_inv(rhs_interim)
    x_b = np.matmul(Gt_F_G, x_a)
    x_p = gtg_inv(x_b)
    G_xp = np.matmul(G, x_p)
    Finv_G_xp = finv(G_xp)
    return np.concatenate((Finv_v - Finv_G_xp, x_p))


def make_case(prec, utils, tag, n, xi, eta_n, eta_s, c, d, big=False):
    bp = prec.MultiphaseBlockPreconditioner(n, xi, eta_n, eta_s)
    A, S, F, D, G = bp.get_big_A_matrix(c=c, d_u=d)
    out = {"params": np.array([n, xi, eta_n, eta_s, c, d, 1.0, -1.0])}
    out.update(csr_fields("A", A))
    if tag == "const75":
        out["theta_const"] = np.array(THETA_CONST)
        u_vec, b_vec = manufactured_const75(n, c, d, xi, eta_n, eta_s, utils)
    else:
        u_vec, b_vec = manufactured(n, c, d, xi, eta_n, eta_s, utils)
    out["u_vec"], out["b_vec"] = u_vec, b_vec
    out["Au"] = np.matmul(A, u_vec)                                  # apply.py:72
    if not big:
        for tag_b, is_ths in (("n", False), ("s", True)):
            L, Dp, XI, Gp = bp.get_block_matrices(is_ths=is_ths)
            out.update(csr_fields("L" + tag_b, L))
            out.update(csr_fields("D" + tag_b, Dp))
            out.update(csr_fields("XI" + tag_b, XI))
            out.update(csr_fields("G" + tag_b, Gp))
        out.update(csr_fields("F", F))
        out.update(csr_fields("D", D))
        out.update(csr_fields("G", G))
        mD = -1.0 * D                                                # solve.py:246-249
        Gt_G = np.matmul(mD, G)
        Gt_F = np.matmul(mD, F)
        Gt_F_G = np.matmul(Gt_F, G)
        out.update(csr_fields("GtG", Gt_G))
        out.update(csr_fields("GtFG", Gt_F_G))
        if n <= 8:
            out["S"] = S
        rng = np.random.default_rng(1234 + n)
        v = rng.standard_normal(A.shape[0])
        out["v"] = v
        # (a) exact inner inverses: F solved exactly, the singular Gt_G by its pseudo-inverse
        GtG_pinv = np.linalg.pinv(Gt_G)
        out["schur_exact"] = approx_schur(F, D, G, v, lambda r: np.linalg.solve(F, r),
                                          lambda r: GtG_pinv @ r, Gt_F_G)
        # (b) Jacobi inner solves, N sweeps from x = 0 (solve.py:149, 262/268 commented path)
        for nf, npp in ((1, 1), (3, 2)):
            out[f"schur_jacobi_{nf}_{npp}"] = approx_schur(
                F, D, G, v, lambda r: jacobi(F, r, nf, 0 * r), lambda r: jacobi(Gt_G, r, npp, 0 * r), Gt_F_G)
        out["jacobi_F_4"] = jacobi(F, v[:F.shape[0]], 4, 0 * v[:F.shape[0]])
        out["jacobi_GtG_4"] = jacobi(Gt_G, v[F.shape[0]:], 4, 0 * v[F.shape[0]:])
    path = os.path.join(HERE, f"golden_n{n}_{tag}.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    prec, utils = load_reference(ref)
    for case in CASES:
        make_case(prec, utils, *case)
    for case in BIG:
        make_case(prec, utils, *case, big=True)
    # the constant-thn cases run the reference's assembly with its module-level thn (which ths and
    # get_thn_vals / get_big_A_matrix look up at call time) bound to the constant
    variable_thn = prec.thn
    prec.thn = lambda y, x: THETA_CONST
    try:
        for *case, big in CONST:
            make_case(prec, utils, *case, big=big)
    finally:
        prec.thn = variable_thn


if __name__ == "__main__":
    main()
