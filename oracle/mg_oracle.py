"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the geometric multigrid inner solve (mp-block-preconditioners_amd/mg.py).

The reference has no multigrid code: its inner inverses are ilupp ILUT factorizations (solve.py:250-254), and
its comments name multigrid as the production choice ("In IBAMR, we'd use Multigrid PC with Jacobi smoother",
solve.py:266, 274).  This module restates the GPU hierarchy and V-cycle from their definitions, so the GPU
results can be checked bit for bit:

* ``p1d`` / ``transfer``: linear interpolation per axis (cell- or node-centred), P as a Kronecker product,
  R = P^T (numpy / scipy construction, independent of the HIP kernel);
* ``hierarchy``: Galerkin coarse operators R (A P) by ``csr_oracle.spgemm`` (sequential C);
* ``vcycle`` / ``mg_solve``: Chebyshev-Jacobi smoothing by ``csr_oracle.cheb_init`` / ``cheb_step``, residual,
  restriction and prolongation by ``csr_oracle.spmv`` -- the GPU's operation order.

Parity pinning: there is nothing in the reference to pin a multigrid cycle against, so this restatement is
"parity unpinned" with respect to the reference (its operators, the pieces it composes, are pinned by
tests/test_oracle_golden.py); the GPU cycle is pinned to this restatement bit for bit.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

from . import csr_oracle as co
from .schur_oracle import cheb_coeffs, gershgorin

CELL, NODE = 0, 1
FIELDS_VELOCITY = ((CELL, NODE), (NODE, CELL), (CELL, NODE), (NODE, CELL))
FIELDS_PRESSURE = ((CELL, CELL),)
COARSE_RCOND = 1e-11   # the coarsest operator's null-space cut (mg.py COARSE_RCOND: Gt_G's constant mode is roundoff)


def p1d(nf: int, kind: int) -> sp.csr_matrix:
    """1D linear interpolation, periodic, fine size nf -> coarse nf / 2."""
    nc = nf // 2
    i = np.arange(nc)
    if kind == CELL:   # fine 2i at 3/4 c_i + 1/4 c_{i-1}; fine 2i+1 at 3/4 c_i + 1/4 c_{i+1}
        R = np.concatenate([2 * i, 2 * i, 2 * i + 1, 2 * i + 1])
        C = np.concatenate([i, (i - 1) % nc, i, (i + 1) % nc])
        V = np.concatenate([np.full(nc, 0.75), np.full(nc, 0.25), np.full(nc, 0.75), np.full(nc, 0.25)])
    else:              # fine 2i on c_i; fine 2i+1 halfway to c_{i+1}
        R = np.concatenate([2 * i, 2 * i + 1, 2 * i + 1])
        C = np.concatenate([i, i, (i + 1) % nc])
        V = np.concatenate([np.ones(nc), np.full(nc, 0.5), np.full(nc, 0.5)])
    M = sp.csr_matrix((V, (R, C)), shape=(nf, nc))
    M.sort_indices()
    return M


def transfer(n: int, fields, which: str) -> sp.csr_matrix:
    """which 'P' (fine x coarse) or 'R' (= P^T) for stacked fields of an n x n grid."""
    P = sp.block_diag([sp.kron(p1d(n, ky), p1d(n, kx)) for ky, kx in fields], format="csr")
    P.eliminate_zeros()   # scipy's kron may store a small dense block's zeros; P has no structural zeros
    M = P if which == "P" else P.T.tocsr()
    M = sp.csr_matrix(M)
    M.sort_indices()
    return M


def hierarchy(A: sp.csr_matrix, n: int, fields, coarsest: int = 8):
    """[(A_l, n_l)], [P_l], [R_l] of the Galerkin hierarchy (same stopping rule as mg.Multigrid: coarsen by 2
    until n <= coarsest, but at least once)."""
    ops, Ps, Rs = [(sp.csr_matrix(A), n)], [], []
    m = n
    while not (m % 2 or (m <= coarsest and len(ops) > 1) or m // 2 < 2):
        P, R = transfer(m, fields, "P"), transfer(m, fields, "R")
        A = co.spgemm(R, co.spgemm(A, P))
        Ps.append(P)
        Rs.append(R)
        m //= 2
        ops.append((A, m))
    return ops, Ps, Rs


def smooth(A, diag, lmin, lmax, K, b, x=None, sub=None):
    """K Chebyshev-Jacobi sweeps from x (None: from 0, first sweep = init pass); sub - x on the last."""
    c1, c2 = cheb_coeffs(lmin, lmax, K)
    d = np.zeros(A.shape[0])
    s = 0
    if x is None:
        x = co.cheb_init(b, diag, c2[0], d, sub if K == 1 else None)
        s = 1
    for k in range(s, K):
        x = co.cheb_step(A, x, b, diag, c1[k], c2[k], d, sub if k == K - 1 else None)
    return x


class MgOracle:
    """V-cycles over ``hierarchy``.  bounds: per-level (lmin, lmax) (default Gershgorin / ratio); coarse_inv:
    the coarsest level's pseudo-inverse (default numpy pinv with singular values below COARSE_RCOND * sigma_max
    dropped, the product's rule, mg.py COARSE_RCOND)."""

    def __init__(self, A, n, fields, pre=2, post=2, cycles=1, ratio=4.0, coarsest=8, bounds=None, coarse_inv=None):
        self.ops, self.P, self.R = hierarchy(A, n, fields, coarsest)
        self.diags = [np.asarray(M.diagonal(), dtype=np.float64) for M, _ in self.ops]
        if bounds is None:
            bounds = []
            for (M, _), d in zip(self.ops, self.diags):
                lmax = gershgorin(M, d)
                bounds.append((lmax / ratio, lmax))
        self.bounds = bounds
        self.pre, self.post, self.cycles = pre, post, cycles
        Ac = self.ops[-1][0].toarray()
        self.coarse_inv = np.linalg.pinv(Ac, rcond=COARSE_RCOND) if coarse_inv is None else np.asarray(coarse_inv)
        m = self.coarse_inv.shape[0]
        self._cinv = sp.csr_matrix((self.coarse_inv.reshape(-1), np.tile(np.arange(m), m),
                                    np.arange(0, m * m + 1, m)), shape=(m, m))

    def vcycle(self, l, b, x=None, sub=None):
        A, _ = self.ops[l]
        d = self.diags[l]
        lmin, lmax = self.bounds[l]
        x = smooth(A, d, lmin, lmax, self.pre, b, x)
        r = co.spmv(A, x, b, mode=2)
        bc = co.spmv(self.R[l], r)
        if l + 1 == len(self.ops) - 1:
            xc = co.spmv(self._cinv, bc)
        else:
            xc = self.vcycle(l + 1, bc)
        x = co.spmv(self.P[l], xc, x, mode=1)
        return smooth(A, d, lmin, lmax, self.post, b, x, sub)

    def solve(self, b, sub=None):
        b = np.ascontiguousarray(b, dtype=np.float64)
        x = None
        for k in range(self.cycles):
            x = self.vcycle(0, b, x, sub if k == self.cycles - 1 else None)
        return x
