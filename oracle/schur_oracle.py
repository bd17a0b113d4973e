"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the preconditioner apply.

``approx_schur_apply`` restates ``approx_schur_op`` (solve.py:257-277):

    Finv_v      = F_inv @ v[:nu]                       solve.py:258
    rhs_interim = D @ Finv_v + v[nu:]                  solve.py:259
    x_a         = GtG_inv @ rhs_interim                solve.py:265
    x_b         = Gt_F_G @ x_a                         solve.py:267
    x_p         = GtG_inv @ x_b                        solve.py:271
    G_xp        = G @ x_p                              solve.py:273
    u           = Finv_v - F_inv @ G_xp                solve.py:274-275
    return [u, x_p]                                    solve.py:276

The reference's inner inverses are ilupp ILUT factorizations (solve.py:251-254; ilupp 1.0.2,
absent here -- parity of that choice is unpinned).  This oracle provides the inner solvers the
GPU path implements:

* ``Inner("jacobi", k)``      k sweeps of solve.py:149-159's Jacobi from x = 0
* ``Inner("chebyshev", k, lmin, lmax)``  k Chebyshev-Jacobi sweeps (Saad Alg. 12.1)
* ``Inner("exact")``          dense solve / pseudo-inverse (tiny n only; pins the composition
                              against the reference's own matrices)

Each sparse step calls oracle/csr_oracle.c, whose operation order equals the GPU kernels', so
GPU results must match this oracle bit for bit on the same inputs.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import csr_oracle as co


@dataclass
class Inner:
    kind: str = "chebyshev"
    sweeps: int = 4
    lmin: float = 0.0
    lmax: float = 0.0


def cheb_coeffs(lmin, lmax, sweeps):
    """Chebyshev-Jacobi coefficients; same expressions as mpbp.hip cheb_coeffs."""
    theta = (lmax + lmin) / 2.0
    delta = (lmax - lmin) / 2.0
    sigma = theta / delta
    rho = 1.0 / sigma
    c1 = [0.0]
    c2 = [1.0 / theta]
    for _ in range(1, sweeps):
        rho_new = 1.0 / (2.0 * sigma - rho)
        c1.append(rho_new * rho)
        c2.append(2.0 * rho_new / delta)
        rho = rho_new
    return c1, c2


def diagonal(M):
    return np.asarray(M.diagonal(), dtype=np.float64)


def gershgorin(M, diag):
    a = abs(M).tocsr()
    s = np.asarray(a.sum(axis=1)).ravel()
    return float(np.max(s / np.abs(diag)))


def inner_solve(M, diag, inner: Inner, b, sub=None, dense_inv=None):
    """x ~ M^-1 b from x0 = 0; returns sub - x when sub is given."""
    if inner.kind == "exact":
        x = dense_inv(b)
        return x if sub is None else sub - x
    K = inner.sweeps
    if inner.kind == "jacobi":
        x = co.jacobi_init(b, diag, sub if K == 1 else None)
        for s in range(1, K):
            x = co.jacobi_step(M, x, b, diag, sub if s == K - 1 else None)
        return x
    if inner.kind == "chebyshev":
        c1, c2 = cheb_coeffs(inner.lmin, inner.lmax, K)
        d = np.empty(M.shape[0], dtype=np.float64)
        x = co.cheb_init(b, diag, c2[0], d, sub if K == 1 else None)
        for s in range(1, K):
            x = co.cheb_step(M, x, b, diag, c1[s], c2[s], d, sub if s == K - 1 else None)
        return x
    raise ValueError(inner.kind)


def approx_schur_apply(F, D, G, GtG, GtFG, v, inner_F: Inner, inner_P: Inner,
                       diag_F=None, diag_P=None, F_inv=None, GtG_inv=None):
    nu = F.shape[0]
    diag_F = diagonal(F) if diag_F is None else diag_F
    diag_P = diagonal(GtG) if diag_P is None else diag_P
    v = np.ascontiguousarray(v, dtype=np.float64)
    Finv_v = inner_solve(F, diag_F, inner_F, v[:nu], dense_inv=F_inv)
    rhs = co.spmv(D, Finv_v, v[nu:], mode=1)
    x_a = inner_solve(GtG, diag_P, inner_P, rhs, dense_inv=GtG_inv)
    x_b = co.spmv(GtFG, x_a)
    x_p = inner_solve(GtG, diag_P, inner_P, x_b, dense_inv=GtG_inv)
    G_xp = co.spmv(G, x_p)
    u = inner_solve(F, diag_F, inner_F, G_xp, sub=Finv_v, dense_inv=F_inv)
    return np.concatenate([u, x_p])


def _inner_solve_scipy(M, diag, inner: Inner, b, sub=None):
    """inner_solve with scipy.sparse products and numpy vector updates (the reference's own CPU form:
    solve.py:149-159 Jacobi, `A @ x` on scipy CSR); same recurrences and coefficients as inner_solve."""
    K = inner.sweeps
    if inner.kind == "jacobi":
        x = b / diag
        for _ in range(1, K):
            x = x + (b - M @ x) / diag
    elif inner.kind == "chebyshev":
        c1, c2 = cheb_coeffs(inner.lmin, inner.lmax, K)
        d = c2[0] * (b / diag)
        x = d
        for s in range(1, K):
            d = c1[s] * d + c2[s] * ((b - M @ x) / diag)
            x = x + d
    else:
        raise ValueError(inner.kind)
    return x if sub is None else sub - x


def approx_schur_apply_scipy(F, D, G, GtG, GtFG, v, inner_F: Inner, inner_P: Inner, diag_F, diag_P):
    """approx_schur_op (solve.py:257-277) composed from scipy.sparse `@` products, as the reference runs
    it on the CPU.  Used only as bench.py's reported CPU baseline (scipy's summation may contract
    differently from the C restatement: compared within 1e-12, not bit for bit)."""
    nu = F.shape[0]
    Finv_v = _inner_solve_scipy(F, diag_F, inner_F, v[:nu])
    rhs = D @ Finv_v + v[nu:]
    x_a = _inner_solve_scipy(GtG, diag_P, inner_P, rhs)
    x_b = GtFG @ x_a
    x_p = _inner_solve_scipy(GtG, diag_P, inner_P, x_b)
    u = _inner_solve_scipy(F, diag_F, inner_F, G @ x_p, sub=Finv_v)
    return np.concatenate([u, x_p])
