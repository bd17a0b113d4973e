"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference's operator assembly.

Restates ``preconditioner.py`` of the reference (abarret/mp-block-preconditioners):

* ``thn`` / ``ths``                         preconditioner.py:9-15
* ``get_thn_vals``                          preconditioner.py:26-84
* ``get_block_matrices`` (L, D, XI, G)      preconditioner.py:86-297
* ``get_big_A_matrix`` (A, F, D, G)         preconditioner.py:299-341
* the approximate-commutator products       solve.py:246-249 (Gt_G = -D G, Gt_F_G = (-D F) G)

The reference fills dense ``np.zeros`` matrices entry by entry; a later
assignment to the same (row, col) replaces an earlier one (this only happens
for n <= 2, where periodic neighbours coincide).  We restate that as
"last write wins" over the same ordered list of writes and keep every stencil
position as a structural entry of a CSR matrix (the reference has no CSR; its
dense zeros and our structural zeros compare equal in ``tests/``).

``get_thn_vals`` evaluates thn at cell centres with periodic wrap-around; we
evaluate thn once per cell into a table (``theta_tables``) and index it
periodically.  The reference sometimes evaluates the same periodic cell at a
shifted coordinate (e.g. x = -1.5 dx instead of (n-1.5) dx), which changes the
last bit of sin(); the golden-fixture tests therefore compare values with a
1e-12 relative tolerance, while the GPU assembly (fed the same tables) must
match this oracle bit for bit.

Arithmetic is written in the reference's evaluation order (Python is
left-associative, no fused multiply-add), so the composite entries here are the
same IEEE operations the reference performs on the same theta values.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

PI = np.pi


def thn(y, x):
    """Network volume fraction, preconditioner.py:9-11."""
    return 0.25 * np.sin(2 * PI * x) * np.sin(2 * PI * y) + 0.5


def theta_tables(n: int):
    """thn at cell centres, u faces and v faces (grid row r counts downwards, y = -(r+0.5) dy).

    cell[r*n+c]  = thn(-(r+0.5)dy, (c+0.5)dx)   -- get_thn_vals, preconditioner.py:26-72
    uface[r*n+c] = thn(-(r+0.5)dy, c dx)        -- w_thn for u, preconditioner.py:325
    vface[r*n+c] = thn(-r dy, (c+0.5)dx)        -- w_thn for v, preconditioner.py:326
    """
    dx = 1 / n
    dy = 1 / n
    r, c = np.divmod(np.arange(n * n, dtype=np.int64), n)
    cell = thn(-(r + 0.5) * dy, (c + 0.5) * dx)
    uface = thn(-(r + 0.5) * dy, c * dx)
    vface = thn(-r * dy, (c + 0.5) * dx)
    return (np.ascontiguousarray(cell, dtype=np.float64),
            np.ascontiguousarray(uface, dtype=np.float64),
            np.ascontiguousarray(vface, dtype=np.float64))


def _csr_last_wins(nrows, ncols, writes):
    """Build a CSR matrix from an ordered list of (rows, cols, vals) dense assignments."""
    R = np.concatenate([np.asarray(w[0], dtype=np.int64) for w in writes])
    C = np.concatenate([np.asarray(w[1], dtype=np.int64) for w in writes])
    V = np.concatenate([np.broadcast_to(np.asarray(w[2], dtype=np.float64), np.shape(w[0]))
                        for w in writes])
    seq = np.arange(R.size)
    order = np.lexsort((seq, C, R))
    R, C, V = R[order], C[order], V[order]
    keep = np.ones(R.size, dtype=bool)
    keep[:-1] = (R[1:] != R[:-1]) | (C[1:] != C[:-1])   # last write of each (row, col)
    R, C, V = R[keep], C[keep], V[keep]
    indptr = np.zeros(nrows + 1, dtype=np.int64)
    np.cumsum(np.bincount(R, minlength=nrows), out=indptr[1:])
    return sp.csr_matrix((V, C.astype(np.int32), indptr.astype(np.int32)), shape=(nrows, ncols))


class _Grid:
    def __init__(self, n):
        self.n = n
        self.N = n * n
        self.r, self.c = np.divmod(np.arange(self.N, dtype=np.int64), n)

    def idx(self, dr, dc):
        n = self.n
        return ((self.r + dr) % n) * n + (self.c + dc) % n


def phase_blocks(n: int, xi: float, cell: np.ndarray, is_ths: bool):
    """(L, D, XI, G) of one phase as CSR, preconditioner.py:86-297."""
    g = _Grid(n)
    N = g.N
    dx = 1 / n
    dy = 1 / n
    P = (1.0 - cell) if is_ths else cell          # ths_* = 1.0 - thn_*, preconditioner.py:74-81

    def T(dr, dc):
        return P[g.idx(dr, dc)]

    k = np.arange(N, dtype=np.int64)

    # ---- u rows: preconditioner.py:100-179 (u_(i+1/2,j) sits between cells (r,c-1) and (r,c))
    tij, tip1j = T(0, -1), T(0, 0)
    tijp1, tip1jp1 = T(-1, -1), T(-1, 0)
    tijm1, tip1jm1 = T(1, -1), T(1, 0)
    iph_jph = 0.25 * (tij + tijp1 + tip1jp1 + tip1j)
    iph_jmh = 0.25 * (tij + tip1j + tijm1 + tip1jm1)
    iph_j = 0.5 * (tij + tip1j)
    ip1_jph = 0.5 * (tip1j + tip1jp1)
    xi_u = xi * iph_j * (1.0 - iph_j)
    xi_v = xi * ip1_jph * (1.0 - ip1_jph)
    Lw = [
        (k, k, 1 / (dx * dx) * (-tip1j - tij) + 1 / (dy * dy) * (-iph_jph - iph_jmh)),
        (k, N + g.idx(0, 0), 1 / (dx * dy) * (-tip1j + iph_jph)),
        (k, g.idx(0, -1), 1 / (dx * dx) * (tij)),
        (k, g.idx(0, 1), tip1j / (dx * dx)),
        (k, g.idx(-1, 0), 1 / (dy * dy) * (iph_jph)),
        (k, g.idx(1, 0), 1 / (dy * dy) * (iph_jmh)),
        (k, N + g.idx(0, -1), 1 / (dy * dx) * (tij - iph_jph)),
        (k, N + g.idx(1, -1), 1 / (dy * dx) * (iph_jmh - tij)),
        (k, N + g.idx(1, 0), 1 / (dx * dy) * (tip1j - iph_jmh)),
    ]

    # ---- v rows + G + D: preconditioner.py:182-295 (v_(i,j+1/2) sits between cells (r-1,c) and (r,c))
    tij, tip1j = T(0, 0), T(0, 1)
    tijp1, tip1jp1 = T(-1, 0), T(-1, 1)
    tijm1 = T(1, 0)
    tim1j, tim1jp1 = T(0, -1), T(-1, -1)
    imh_jph = 0.25 * (tim1j + tim1jp1 + tij + tijp1)
    iph_jph = 0.25 * (tij + tip1j + tijp1 + tip1jp1)
    i_jph = 0.5 * (tij + tijp1)
    i_jmh = 0.5 * (tij + tijm1)
    imh_j = 0.5 * (tij + tim1j)
    iph_j = 0.5 * (tij + tip1j)
    Gw = [
        (k, k, (1 / dx) * imh_j),
        (k, g.idx(0, -1), -(1 / dx) * imh_j),
        (N + k, k, -(1 / dy) * i_jph),
        (N + k, g.idx(-1, 0), (1 / dy) * i_jph),
    ]
    Dw = [
        (k, g.idx(0, 1), 1 / dx * iph_j),
        (k, k, -1 / dx * imh_j),
        (k, N + k, 1 / dy * i_jph),
        (k, N + g.idx(1, 0), -1 / dy * i_jmh),
    ]
    Lw += [
        (N + k, N + k, -1 / (dy * dy) * (tijp1 + tij) - 1 / (dx * dx) * (iph_jph + imh_jph)),
        (N + k, N + g.idx(0, -1), 1 / (dx * dx) * imh_jph),
        (N + k, N + g.idx(0, 1), 1 / (dx * dx) * iph_jph),
        (N + k, N + g.idx(-1, 0), 1 / (dy * dy) * tijp1),
        (N + k, N + g.idx(1, 0), 1 / (dy * dy) * tij),
        (N + k, k, 1 / (dx * dy) * (imh_jph - tij)),
        (N + k, g.idx(0, 1), 1 / (dy * dx) * (tij - iph_jph)),
        (N + k, g.idx(-1, 0), 1 / (dy * dx) * (tijp1 - imh_jph)),
        (N + k, g.idx(-1, 1), 1 / (dy * dx) * (iph_jph - tijp1)),
    ]
    L = _csr_last_wins(2 * N, 2 * N, Lw)
    D = _csr_last_wins(N, 2 * N, Dw)
    G = _csr_last_wins(2 * N, N, Gw)
    xi_diag = np.concatenate([xi_u, xi_v])
    XI = sp.csr_matrix((xi_diag, np.arange(2 * N, dtype=np.int32), np.arange(2 * N + 1, dtype=np.int32)),
                       shape=(2 * N, 2 * N))
    return L, D, XI, G


def _stack_rows(blocks):
    """Row-wise concatenation of CSR pieces given as (row_offset, col_offset, csr, scale)."""
    R, C, V = [], [], []
    for r0, c0, m, s in blocks:
        coo = m.tocoo()
        R.append(coo.row.astype(np.int64) + r0)
        C.append(coo.col.astype(np.int64) + c0)
        V.append(coo.data if s is None else s * coo.data)
    return np.concatenate(R), np.concatenate(C), np.concatenate(V)


def _csr_from_unique(nrows, ncols, R, C, V):
    order = np.lexsort((C, R))
    R, C, V = R[order], C[order], V[order]
    if R.size > 1:
        assert not np.any((R[1:] == R[:-1]) & (C[1:] == C[:-1])), "duplicate entries"
    indptr = np.zeros(nrows + 1, dtype=np.int64)
    np.cumsum(np.bincount(R, minlength=nrows), out=indptr[1:])
    return sp.csr_matrix((V, C.astype(np.int32), indptr.astype(np.int32)), shape=(nrows, ncols))


class StokesSystem:
    """Oracle for MultiphaseBlockPreconditioner(n, xi, eta_n, eta_s).get_big_A_matrix(c, d_u, d_p, d_div).

    Attributes (CSR, structural stencil pattern, columns sorted):
      A (5N x 5N), F (4N x 4N), D (N x 4N, unscaled hstack(D_n, D_s)), G (4N x N, d_p-scaled),
      GtG = (-D) G, GtFG = ((-D) F) G          (solve.py:246-249)
    with N = n*n and unknown ordering [u_n, v_n, u_s, v_s, p] (preconditioner.py:310-341).
    """

    def __init__(self, n, xi=1.0, eta_n=1.0, eta_s=1.0, c=1.0, d_u=-1.0, d_p=1.0, d_div=-1.0,
                 tables=None, products=True):
        self.n, self.xi, self.eta_n, self.eta_s = n, xi, eta_n, eta_s
        self.c, self.d_u, self.d_p, self.d_div = c, d_u, d_p, d_div
        N = n * n
        self.N = N
        cell, uface, vface = tables if tables is not None else theta_tables(n)
        self.cell, self.uface, self.vface = cell, uface, vface
        Ln, Dn, XIn, Gn = phase_blocks(n, xi, cell, False)
        Ls, Ds, XIs, Gs = phase_blocks(n, xi, cell, True)
        self.blocks = {"n": (Ln, Dn, XIn, Gn), "s": (Ls, Ds, XIs, Gs)}

        # w_thn / w_ths (preconditioner.py:315-329)
        w_n = np.concatenate([c * uface, c * vface])
        w_s = np.concatenate([c * (1.0 - uface), c * (1.0 - vface)])

        # F = XI + d_u * block_diag(eta_n L_n, eta_s L_s)  (preconditioner.py:310, 331-337)
        pieces = []
        for p, (Lp, XIp, wp, eta) in enumerate(((Ln, XIn, w_n, eta_n), (Ls, XIs, w_s, eta_s))):
            coo = Lp.tocoo()
            rr = coo.row.astype(np.int64)
            cc = coo.col.astype(np.int64)
            xid = XIp.diagonal()
            vals = d_u * (eta * coo.data)
            on_diag = rr == cc
            vals = np.where(on_diag, (wp[rr] - d_u * xid[rr]) + vals, vals)
            off = p * 2 * N
            pieces.append((rr + off, cc + off, vals))
            other = (1 - p) * 2 * N
            ii = np.arange(2 * N, dtype=np.int64)
            pieces.append((ii + off, ii + other, d_u * xid))
        FR = np.concatenate([q[0] for q in pieces])
        FC = np.concatenate([q[1] for q in pieces])
        FV = np.concatenate([q[2] for q in pieces])
        self.F = _csr_from_unique(4 * N, 4 * N, FR, FC, FV)

        # D = hstack(D_n, D_s), G = vstack(d_p G_n, d_p G_s)  (preconditioner.py:311-313)
        self.D = _csr_from_unique(N, 4 * N, *_stack_rows([(0, 0, Dn, None), (0, 2 * N, Ds, None)]))
        self.G = _csr_from_unique(4 * N, N, *_stack_rows([(0, 0, Gn, d_p), (2 * N, 0, Gs, d_p)]))

        # A = [[F, G], [d_div D, 0]]  (preconditioner.py:339-341)
        fc = self.F.tocoo()
        gc = self.G.tocoo()
        dc = self.D.tocoo()
        AR = np.concatenate([fc.row.astype(np.int64), gc.row.astype(np.int64),
                             dc.row.astype(np.int64) + 4 * N])
        AC = np.concatenate([fc.col.astype(np.int64), gc.col.astype(np.int64) + 4 * N,
                             dc.col.astype(np.int64)])
        AV = np.concatenate([fc.data, gc.data, d_div * dc.data])
        self.A = _csr_from_unique(5 * N, 5 * N, AR, AC, AV)

        if products:
            from . import csr_oracle as co
            # Gt_G = (-1.0 * D) @ G ; Gt_F_G = ((-1.0 * D) @ F) @ G   (solve.py:246-249)
            self.GtG = co.spgemm(self.D, self.G, alpha=-1.0)
            GtF = co.spgemm(self.D, self.F, alpha=-1.0)
            self.GtFG = co.spgemm(GtF, self.G, alpha=1.0)

    def block_matrices(self, is_ths):
        """(L, D, XI, G) of one phase, mirrors get_block_matrices(is_ths) (preconditioner.py:86)."""
        return self.blocks["s" if is_ths else "n"]
