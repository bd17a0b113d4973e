"""MultiphaseBlockPreconditioner -- the reference's operator-assembly interface, assembled in HBM.

Mirrors ``preconditioner.py`` of abarret/mp-block-preconditioners:

    thn(y, x), ths(y, x)                         preconditioner.py:9-15
    MultiphaseBlockPreconditioner(n, xi, eta_n, eta_s)              :17-24
    .get_block_matrices(is_ths) -> (L, D, XI, G)                     :86-297
    .get_big_A_matrix(c, d_u, d_p=1.0, d_div=-1.0) -> (A, S, F, D, G) :299-349

Every matrix is a ``DeviceCSR`` built on the GPU by the stencil kernels of libmpbp (one thread per
row, last-write-wins over the reference's ordered dense assignments, columns sorted).  The
reference also returns the exact Schur complement S = -D F^-1 G (a dense inverse, O(N^3)); that
is not formed here (``S`` is None) -- the approximate-commutator preconditioner in
``solve.ApproxSchurPreconditioner`` is the path the reference actually solves with.
"""
from __future__ import annotations

import ctypes
import weakref

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_handle
from .csr import DeviceCSR, csr_from_row_nnz, spgemm

PI = np.pi


def thn(y, x):
    """Network volume fraction (host helper, preconditioner.py:9-11)."""
    return 0.25 * np.sin(2 * PI * x) * np.sin(2 * PI * y) + 0.5


def ths(y, x):
    """Solvent volume fraction (preconditioner.py:13-15)."""
    return 1.0 - thn(y, x)


class FStencil:
    """What the matrix-free F kernels need: the assembly parameters and the thn tables (HBM)."""

    def __init__(self, prm: _lib.StokesParams, tables):
        self.prm = prm
        self.cell, self.uface, self.vface = tables

    def matvec(self, x, out=None, mode=_lib.SPMV_STORE, z=None, numerics="exact"):
        """y = F x (mode STORE), F x + z (ADD) or z - F x (RESID); numerics 'fast': the tolerance-mode rows."""
        if out is None:
            out = torch.empty(4 * self.prm.n * self.prm.n, dtype=torch.float64, device=x.device)
        if numerics not in ("exact", "fast"):
            raise ValueError("numerics must be 'exact' or 'fast'")
        mode = int(mode) | (_lib.SPMV_FAST if numerics == "fast" else 0)
        check(lib().mpbp_f_stencil_spmv(ctypes.byref(self.prm), ptr(self.cell), ptr(self.uface), ptr(self.vface),
                                        None, mode, ptr(x), ptr(z), ptr(out), stream_handle()))
        return out


class PGStencil:
    """Matrix-free D, G or Gt_G = -(D G) (op = _lib.PG_D / PG_G / PG_GTG), recomputed per row from the cell
    thn table -- bit-identical to the assembled operator (and, for Gt_G, to the sparse product)."""

    def __init__(self, prm: _lib.StokesParams, cell: torch.Tensor, op: int):
        self.prm, self.cell, self.op = prm, cell, int(op)

    @property
    def shape(self):
        N = self.prm.n * self.prm.n
        return {_lib.PG_D: (N, 4 * N), _lib.PG_G: (4 * N, N), _lib.PG_GTG: (N, N)}[self.op]

    def same_grid(self, other) -> bool:
        """True when `other` was built from the same tables and parameters (one get_big_A_matrix call)."""
        return isinstance(other, (PGStencil, FStencil)) and other.cell.data_ptr() == self.cell.data_ptr() and \
            bytes(other.prm) == bytes(self.prm)

    def matvec(self, x, out=None, mode=_lib.SPMV_STORE, z=None):
        if out is None:
            out = torch.empty(self.shape[0], dtype=torch.float64, device=x.device)
        check(lib().mpbp_pg_stencil_spmv(ctypes.byref(self.prm), ptr(self.cell), None, self.op, mode, ptr(x), ptr(z),
                                         ptr(out), stream_handle()))
        return out


class MultiphaseBlockPreconditioner:
    def __init__(self, n, xi, eta_n=1.0, eta_s=1.0, device=None):
        if int(n) < 1:
            raise ValueError("n must be >= 1")
        self.n = int(n)
        self.dx = 1 / self.n
        self.dy = 1 / self.n
        self.xi = float(xi)
        self.eta_n = float(eta_n)
        self.eta_s = float(eta_s)
        self.device = torch.device(device or "cuda")
        self._theta = None

    # -- volume fraction tables (HBM) ---------------------------------------------------------------
    def theta_tables(self):
        """(cell, uface, vface) thn tables, n*n each, computed on the GPU."""
        if self._theta is None:
            N = self.n * self.n
            t = [torch.empty(N, dtype=torch.float64, device=self.device) for _ in range(3)]
            check(lib().mpbp_stokes_theta(self.n, ptr(t[0]), ptr(t[1]), ptr(t[2]), stream_handle()))
            self._theta = tuple(t)
        return self._theta

    def set_theta_tables(self, cell, uface, vface):
        """Use caller-provided thn tables (any volume-fraction field; host arrays or tensors of n*n values, or
        scalars for a constant thn such as BASELINE configs[0]'s / solve.py:60-68's 0.75)."""
        N = self.n * self.n
        tabs = []
        for a in (cell, uface, vface):
            if np.ndim(a) == 0 and not isinstance(a, torch.Tensor):
                a = np.full(N, float(a))
            a = torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64) if isinstance(a, np.ndarray) else a)
            a = a.to(device=self.device, dtype=torch.float64).contiguous()
            if a.numel() != N:
                raise ValueError("theta tables must have n*n entries")
            tabs.append(a)
        self._theta = tuple(tabs)

    def _params(self, c=1.0, d_u=-1.0, d_p=1.0, d_div=-1.0):
        return _lib.StokesParams(self.n, self.xi, self.eta_n, self.eta_s, float(c), float(d_u), float(d_p),
                                 float(d_div))

    def assemble(self, op, c=1.0, d_u=-1.0, d_p=1.0, d_div=-1.0) -> DeviceCSR:
        cell, uface, vface = self.theta_tables()
        prm = self._params(c, d_u, d_p, d_div)
        rows = check(lib().mpbp_stokes_rows(self.n, op))
        cols = check(lib().mpbp_stokes_cols(self.n, op))
        row_nnz = torch.empty(rows, dtype=torch.int32, device=self.device)
        check(lib().mpbp_stokes_count(ctypes.byref(prm), op, ptr(cell), ptr(row_nnz), stream_handle()))
        rp, ci, va = csr_from_row_nnz(row_nnz, (rows, cols), self.device)
        check(lib().mpbp_stokes_fill(ctypes.byref(prm), op, ptr(cell), ptr(uface), ptr(vface), ptr(rp), ptr(ci),
                                     ptr(va), stream_handle()))
        return DeviceCSR(rp, ci, va, (rows, cols))

    def assemble_rows(self, op, rows: torch.Tensor, global_shape: bool = False, c=1.0, d_u=-1.0, d_p=1.0,
                      d_div=-1.0) -> DeviceCSR:
        """Rows `rows` (ascending global ids, device int32) of operator `op` with their global columns -- the
        global assembly's rows bit for bit (mpbp_stokes_count_rows / _fill_rows) without assembling the others (a
        rank's owned and ghost rows, preconditioner.py:299-341).  global_shape: the result has every row of the
        operator, those outside `rows` empty (an operand a sparse product indexes by global row)."""
        cell, uface, vface = self.theta_tables()
        prm = self._params(c, d_u, d_p, d_div)
        nglob = check(lib().mpbp_stokes_rows(self.n, op))
        cols = check(lib().mpbp_stokes_cols(self.n, op))
        rows = rows.to(device=self.device, dtype=torch.int32).contiguous()
        m = rows.numel()
        row_nnz = torch.empty(max(m, 1), dtype=torch.int32, device=self.device)[:m]
        check(lib().mpbp_stokes_count_rows(ctypes.byref(prm), op, ptr(cell), ptr(rows), m, ptr(row_nnz),
                                           stream_handle()))
        rp, ci, va = csr_from_row_nnz(row_nnz, (m, cols), self.device)
        check(lib().mpbp_stokes_fill_rows(ctypes.byref(prm), op, ptr(cell), ptr(uface), ptr(vface), ptr(rows), m,
                                          ptr(rp), ptr(ci), ptr(va), stream_handle()))
        if not global_shape:
            return DeviceCSR(rp, ci, va, (m, cols))
        if m > 1 and not bool((rows[1:] > rows[:-1]).all()):
            raise ValueError("assemble_rows(global_shape=True) needs ascending rows")
        counts = torch.zeros(nglob, dtype=torch.int64, device=self.device)
        counts[rows.long()] = (rp[1:] - rp[:-1]).long()
        grp = torch.zeros(nglob + 1, dtype=torch.int64, device=self.device)
        torch.cumsum(counts, 0, out=grp[1:])
        return DeviceCSR(grp.to(torch.int32), ci, va, (nglob, cols))

    def stencils(self, c=1.0, d_u=-1.0, d_p=1.0, d_div=-1.0):
        """(F, D, G) matrix-free forms (FStencil, PGStencil, PGStencil) without assembling the matrices (n >= 3)."""
        if self.n < 3:
            return None, None, None
        prm, tabs = self._params(c, d_u, d_p, d_div), self.theta_tables()
        return FStencil(prm, tabs), PGStencil(prm, tabs[0], _lib.PG_D), PGStencil(prm, tabs[0], _lib.PG_G)

    # -- the reference's interface ---------------------------------------------------------------
    def get_block_matrices(self, is_ths):
        """(L, D, XI, G) of one phase (preconditioner.py:86-297)."""
        s = bool(is_ths)
        return (self.assemble(_lib.OP_L_S if s else _lib.OP_L_N),
                self.assemble(_lib.OP_D_S if s else _lib.OP_D_N),
                self.assemble(_lib.OP_XI_S if s else _lib.OP_XI_N),
                self.assemble(_lib.OP_G_S if s else _lib.OP_G_N))

    def get_big_A_matrix(self, c, d_u, d_p: float = 1.0, d_div: float = -1.0):
        """(A, S, F, D, G) (preconditioner.py:299-349); S (dense exact Schur complement) is None."""
        kw = dict(c=c, d_u=d_u, d_p=d_p, d_div=d_div)
        A = self.assemble(_lib.OP_A, **kw)
        F = self.assemble(_lib.OP_F, **kw)
        D = self.assemble(_lib.OP_D, **kw)
        G = self.assemble(_lib.OP_G, **kw)
        A.row_groups, F.row_groups, G.row_groups = 5, 4, 4   # [u_n|v_n|u_s|v_s|p] rows over the same cells
        if self.n >= 3:   # the matrix-free forms (periodic neighbours are distinct from n = 3 on)
            prm, tabs = self._params(**kw), self.theta_tables()
            F.stencil = FStencil(prm, tabs)
            D.stencil = PGStencil(prm, tabs[0], _lib.PG_D)
            G.stencil = PGStencil(prm, tabs[0], _lib.PG_G)
        return A, None, F, D, G

    @staticmethod
    def commutator_products(F: DeviceCSR, D: DeviceCSR, G: DeviceCSR):
        """Gt_G = (-D) G and Gt_F_G = ((-D) F) G (solve.py:246-249), sparse products in HBM."""
        GtG = spgemm(D, G, alpha=-1.0)
        GtF = spgemm(D, F, alpha=-1.0)
        GtFG = spgemm(GtF, G, alpha=1.0)
        del GtF
        # provenance: the matrix-free Gt_F_G apply (kernel option q13_mf) may stand in for this product only when it
        # IS the product of the operators the preconditioner holds (weak references: the tag keeps nothing alive)
        GtFG._product_of = tuple(weakref.ref(M) for M in (F, D, G))
        sd, sg = getattr(D, "stencil", None), getattr(G, "stencil", None)
        if isinstance(sd, PGStencil) and sd.op == _lib.PG_D and isinstance(sg, PGStencil) and sg.op == _lib.PG_G \
                and sd.same_grid(sg):
            GtG.stencil = PGStencil(sd.prm, sd.cell, _lib.PG_GTG)
        return GtG, GtFG
