"""Geometric multigrid for the inner inverses F^-1 and Gt_G^-1 of the approximate Schur preconditioner.

The reference approximates both inverses with ILUT (solve.py:250-254) and names the scalable choice in
its own comments: "In IBAMR, we'd use Multigrid PC with Jacobi smoother" (solve.py:266, 274).  This is
that choice on the GPU:

* levels: the periodic n x n MAC grid coarsened by 2 per direction down to n <= ``coarsest`` (at least once;
  odd n stops);
* transfers: per field, linear interpolation along each axis -- cell-centred (p; u along y; v along x)
  or node-centred (u along x, v along y) -- as CSR P, and R = P^T (``mpbp_mg_transfer_*``, exact values);
* coarse operators: Galerkin A_{l+1} = R (A_l P) with the library's SpGEMM (every product kept);
* smoother: Chebyshev-Jacobi on [lmax / ratio, lmax] with lmax the Gershgorin bound of diag(A)^-1 A;
* coarsest level: its dense pseudo-inverse (computed once on the host), applied by a dense kernel (one row per
  lane, the CSR row's order) from a column-major copy;
* layouts: every level's operator and transfers also get a SELL-64 copy when their rows fit (< 256 entries):
  the Galerkin coarse operators' long uniform rows (20-50 entries) stream at HBM speed one row per lane, where
  the CSR kernel's per-wave chunks serve rows of <= 12 entries (same bits either way).

``Multigrid.solve`` runs ``cycles`` V-cycles from x = 0 through ``mpbp_mg_solve`` (graph-capturable).
Inside ``ApproxSchurPreconditioner`` (``InnerSolver("mg", cycles)``) level 0 is the apply's own F / Gt_G
operator -- matrix-free when the plan is -- with the same bits.  oracle/mg_oracle.py restates the cycle.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_handle
from .csr import DeviceCSR, DeviceSELL, csr_from_row_nnz, spgemm

CELL, NODE = _lib.MG_CELL, _lib.MG_NODE
# (row axis, column axis) kinds of [u_n, v_n, u_s, v_s]: u at (-(r+1/2) dy, c dx), v at (-r dy, (c+1/2) dx)
# (utils.fill_sol_and_RHS_vecs), p at cell centres
FIELDS_VELOCITY = ((CELL, NODE), (NODE, CELL), (CELL, NODE), (NODE, CELL))
FIELDS_PRESSURE = ((CELL, CELL),)


def transfer(n: int, fields, which: int, device) -> DeviceCSR:
    """P (which = MG_P: fine x coarse) or R = P^T (MG_R) of the n x n grid, built on the GPU."""
    kinds = np.ascontiguousarray(np.asarray(fields, dtype=np.int32).reshape(-1))
    nf = len(fields)
    rows = nf * (n * n if which == _lib.MG_P else (n // 2) ** 2)
    cols = nf * ((n // 2) ** 2 if which == _lib.MG_P else n * n)
    row_nnz = torch.empty(rows, dtype=torch.int32, device=device)
    check(lib().mpbp_mg_transfer_count(n, nf, kinds.ctypes.data_as(ctypes.c_void_p), which, ptr(row_nnz),
                                       stream_handle()))
    rp, ci, va = csr_from_row_nnz(row_nnz, (rows, cols), device)
    check(lib().mpbp_mg_transfer_fill(n, nf, kinds.ctypes.data_as(ctypes.c_void_p), which, ptr(rp), ptr(ci),
                                      ptr(va), stream_handle()))
    return DeviceCSR(rp, ci, va, (rows, cols))


def transfer_rows(n: int, fields, which: int, rows: torch.Tensor) -> DeviceCSR:
    """Rows `rows` (device int32 global ids) of transfer(n, fields, which) with their global columns, the same entries
    (mpbp_mg_transfer_rows_*): a rank's band of a row-partitioned hierarchy."""
    kinds = np.ascontiguousarray(np.asarray(fields, dtype=np.int32).reshape(-1))
    nf = len(fields)
    cols = nf * ((n // 2) ** 2 if which == _lib.MG_P else n * n)
    rows = rows.to(torch.int32).contiguous()
    m = rows.numel()
    nrows = nf * (n * n if which == _lib.MG_P else (n // 2) ** 2)
    if m and (int(rows.min()) < 0 or int(rows.max()) >= nrows):   # the kernel derives (field, row, column) from the id
        raise ValueError(f"transfer_rows: row ids must lie in [0, {nrows}) for {nf} fields of the {n}^2 level")
    row_nnz = torch.empty(max(m, 1), dtype=torch.int32, device=rows.device)[:m]
    check(lib().mpbp_mg_transfer_rows_count(n, nf, kinds.ctypes.data_as(ctypes.c_void_p), which, ptr(rows), m,
                                            ptr(row_nnz), stream_handle()))
    rp, ci, va = csr_from_row_nnz(row_nnz, (m, cols), rows.device)
    check(lib().mpbp_mg_transfer_rows_fill(n, nf, kinds.ctypes.data_as(ctypes.c_void_p), which, ptr(rows), m, ptr(rp),
                                           ptr(ci), ptr(va), stream_handle()))
    return DeviceCSR(rp, ci, va, (m, cols))


def sell_copy(A: DeviceCSR) -> DeviceSELL | None:
    """SELL-64 copy of A when every row has < 256 entries (the layout's row-length byte), else None."""
    rp = A.row_ptr_host
    if A.shape[0] == 0 or int(np.max(np.diff(rp))) > 255:
        return None
    return A.to_sell()


class StencilValues:
    """Stencil-values layout (``mpbp_svl``) of a translation-invariant operator on nf stacked m x m periodic fields: every
    row of field f holds the same K (field, dr, dc) offsets, so only the values are kept, slot-major, and the kernel
    rebuilds an interior row's columns as row + delta[f][s].  Built on the GPU from the CSR arrays (``build``), which it
    verifies: uniform row length, every row's wrapped offsets a permutation of the field's K slots, interior rows in
    slot order (so the interior sums are the CSR row's, bit for bit).  Rows within `reach` of the periodic edge are
    listed for the kernel's CSR path.  None when the operator is not of that form."""

    def __init__(self, A: DeviceCSR, nf: int, m: int, reach: int, K: int, delta, vals, edge_rows):
        self.A, self.nf, self.m, self.reach, self.slots = A, nf, m, reach, K
        self.delta, self.vals, self.edge_rows = delta, vals, edge_rows
        self._cs = _lib.Svl(nf, m, reach, K, delta.data_ptr(), vals.data_ptr(),
                            edge_rows.data_ptr() if edge_rows.numel() else None, int(edge_rows.numel()), 0)

    def cstruct(self):
        return self._cs

    @classmethod
    def build(cls, A: DeviceCSR, nf: int, m: int) -> "StencilValues | None":
        if A.shape != (nf * m * m, nf * m * m) or A.nnz == 0:
            return None
        arrays = stencil_values_arrays(A.row_ptr, A.col_idx, A.val, nf, m)
        return None if arrays is None else cls(A, nf, m, *arrays)

    def matvec(self, x: torch.Tensor, out: torch.Tensor | None = None, mode=_lib.SPMV_STORE,
               z: torch.Tensor | None = None) -> torch.Tensor:
        if out is None:
            out = torch.empty(self.A.shape[0], dtype=torch.float64, device=self.A.device)
        check(lib().mpbp_svl_spmv(ctypes.byref(self._cs), ctypes.byref(self.A.cstruct()), mode, ptr(x), ptr(z),
                                  ptr(out), stream_handle()))
        return out


def stencil_values_arrays(row_ptr: torch.Tensor, col_idx: torch.Tensor, val: torch.Tensor, nf: int, m: int):
    """(reach, K, delta[nf * K], vals[K * N] slot-major, edge_rows) of StencilValues from CSR arrays (any torch device),
    or None when the operator is not translation-invariant in that sense (see StencilValues)."""
    N = nf * m * m
    if row_ptr.numel() != N + 1 or m < 4:
        return None
    dev = row_ptr.device
    rp = row_ptr.long()
    lens = rp[1:] - rp[:-1]
    K = int(lens[0])
    if K < 1 or nf * K > 256 or not bool(torch.all(lens == K)):
        return None
    e = torch.arange(col_idx.numel(), device=dev)
    rows, pos = e // K, e % K
    del e
    mm = m * m
    ci = col_idx.long()
    f, cell = rows // mm, rows % mm
    r, c = cell // m, cell % m
    fc, cc = ci // mm, ci % mm
    dr = (cc // m - r + m // 2) % m - m // 2
    dc = (cc % m - c + m // 2) % m - m // 2
    del cell, cc
    R = int(torch.maximum(dr.abs().max(), dc.abs().max()))
    if m % 2 or m < 2 * R + 4 or K * N > 2 ** 31 - 1:
        return None
    w = 2 * R + 1
    table = torch.full((nf, nf, w, w), -1, dtype=torch.long, device=dev)
    delta = torch.empty(nf, K, dtype=torch.int32, device=dev)
    for f0 in range(nf):
        base = f0 * mm + (m // 2) * m + m // 2
        sl = slice(base * K, base * K + K)
        table[f0, fc[sl], dr[sl] + R, dc[sl] + R] = torch.arange(K, device=dev)
        delta[f0] = (ci[sl] - base).to(torch.int32)
    slot = table[f, fc, dr + R, dc + R]
    del fc, dr, dc, table
    if bool((slot < 0).any()):
        return None
    seen = torch.bincount(rows * K + slot, minlength=N * K)
    if not bool(torch.all(seen == 1)):
        return None
    del seen
    if bool(((slot != pos) & (r >= R) & (r < m - R) & (c >= R) & (c < m - R)).any()):
        return None
    R += R & 1   # the kernel's interior cells go in pairs from an even column: an odd reach widens the edge band
    interior = (r >= R) & (r < m - R) & (c >= R) & (c < m - R)
    vals = torch.empty(K * N, dtype=torch.float64, device=dev)
    vals[slot * N + rows] = val
    row_int = interior.view(N, K)[:, 0]
    edge = torch.nonzero(~row_int).reshape(-1).to(torch.int32)
    return R, K, delta.reshape(-1).contiguous(), vals, edge


def set_transfer_kinds(mg_struct, fields, n0: int):
    """mpbp_mg.tr_*: the transfers' field kinds and level 0's grid size (matrix-free whole-grid transfers)."""
    mg_struct.tr_nfields = len(fields)
    mg_struct.tr_n0 = int(n0)
    for f, (ky, kx) in enumerate(fields):
        mg_struct.tr_ky[f] = ky
        mg_struct.tr_kx[f] = kx


SVL_MIN_ROWS = 65536     # Multigrid's default: levels >= 1 above this many rows get a stencil-values copy
MAX_COARSE_ROWS = 8192   # the coarsest level's dense pseudo-inverse: 8192^2 doubles = 512 MB, an O(m^3) host pinv
# Singular values below COARSE_RCOND * sigma_max of the coarsest operator are its null space.  Gt_G on the periodic
# grid annihilates constants; after six Galerkin products that mode's singular value is roundoff, 8.5e-16 sigma_max at
# 256^2 but 5.6e-15 at 1024^2 -- above numpy's default cut (1e-15), so the pseudo-inverse inverted it and the pressure
# solve's output carried a ~1e17 constant.  The next singular values are 9e-2 (Gt_G) and, for F, 7.5e-6 (eta ratio
# 100) / 7.5e-8 (10^4) (tools/coarse_spectrum.py): 1e-11 sits orders of magnitude from both.
COARSE_RCOND = 1e-11


def dense_inverse_csr(A: DeviceCSR) -> tuple[DeviceCSR, np.ndarray]:
    """The pseudo-inverse of a small operator as a CSR with every entry stored (rows of ncols entries)."""
    if A.shape[0] > MAX_COARSE_ROWS:
        raise ValueError(f"coarsest level has {A.shape[0]} rows (> {MAX_COARSE_ROWS}): its dense pseudo-inverse would "
                         f"need {A.shape[0] ** 2 * 8 / 1e9:.1f} GB and an O(m^3) factorisation; coarsening stops at an odd "
                         "grid size, so use a grid n = m 2^k with a small m (or a larger `coarsest`)")
    Ad = A.to_scipy().toarray()
    inv = np.ascontiguousarray(np.linalg.pinv(Ad, rcond=COARSE_RCOND))
    m = inv.shape[0]
    dev = A.device
    rp = np.arange(0, m * m + 1, m, dtype=np.int32)
    ci = np.tile(np.arange(m, dtype=np.int32), m)
    M = DeviceCSR(torch.from_numpy(rp).to(dev), torch.from_numpy(ci).to(dev),
                  torch.from_numpy(inv.reshape(-1).copy()).to(dev), (m, m), row_ptr_host=rp)
    return M, inv


def level_sizes(n: int, coarsest: int) -> list[int]:
    """Grid sizes of the hierarchy: halve while even, down to <= coarsest (at least one coarsening)."""
    sizes = [n]
    m = n
    while not (m % 2 or (m <= coarsest and len(sizes) > 1) or m // 2 < 2):
        m //= 2
        sizes.append(m)
    return sizes


class Multigrid:
    """V-cycle hierarchy over a stacked-field operator A (DeviceCSR) of an n x n periodic grid.

    fields   per stacked field, the (row axis, column axis) kinds -- FIELDS_VELOCITY for F, FIELDS_PRESSURE
             for Gt_G
    pre/post Chebyshev-Jacobi smoothing sweeps per level; ratio: lmin = lmax / ratio
    cycles   V-cycles per solve (x0 = 0); coarsest: stop coarsening at n <= coarsest
    sell     SELL-64 copies of the operators / transfers and the dense coarse kernel (False: CSR throughout)
    fine_sell  also a SELL copy of level 0's operator (the standalone solve's fine level)
    svl_min_rows  levels >= 1 with more rows get a stencil-values copy (StencilValues; None: never) -- used where the
             grouped small-level kernel is not (kernel option mg_group_rows)
    kernel_opts  overrides of the process-default kernel choices for this hierarchy's standalone solve (_lib.KernelOpts
             field names)
    """

    def __init__(self, A: DeviceCSR, n: int, fields=FIELDS_PRESSURE, pre: int = 2, post: int = 2, cycles: int = 1,
                 ratio: float = 4.0, coarsest: int = 8, diag: torch.Tensor | None = None, sell: bool = True,
                 fine_sell: bool = True, svl_min_rows: int | None | str = "default", kernel_opts: dict | None = None):
        nf = len(fields)
        if A.shape != (nf * n * n, nf * n * n):
            raise ValueError(f"operator {A.shape} is not {nf} fields of a {n} x {n} grid")
        if n < 4 or n % 2 or n // 2 < 2:
            raise ValueError("multigrid needs an even grid n >= 4")
        if pre < 1 or post < 1 or cycles < 1:
            raise ValueError("pre, post and cycles must be >= 1")
        self.n, self.fields, self.pre, self.post, self.cycles, self.ratio = n, tuple(fields), pre, post, cycles, ratio
        self.coarsest = coarsest
        dev = A.device
        self.device = dev
        sizes = level_sizes(n, coarsest)
        if nf * sizes[-1] ** 2 > MAX_COARSE_ROWS:   # refuse before any Galerkin product is formed
            raise ValueError(f"grid {n} coarsens to {sizes} (stopping at an odd size): the coarsest level's "
                             f"{nf * sizes[-1] ** 2} rows exceed the dense inverse's {MAX_COARSE_ROWS}")
        self.ops, self.diags, self.R, self.P, self.bounds, self.sizes = [], [], [], [], [], []
        m = n
        while True:
            d = diag if (not self.ops and diag is not None) else A.diagonal()
            lmax = A.gershgorin(d)
            self.ops.append(A)
            self.diags.append(d)
            self.bounds.append((lmax / ratio, lmax))
            self.sizes.append(m)
            if m % 2 or (m <= coarsest and len(self.ops) > 1) or m // 2 < 2:   # (at least one coarsening)
                break
            P = transfer(m, fields, _lib.MG_P, dev)
            R = transfer(m, fields, _lib.MG_R, dev)
            self.P.append(P)
            self.R.append(R)
            A = spgemm(R, spgemm(A, P))
            m //= 2
        if len(self.ops) < 2:
            raise ValueError(f"grid {n} gives a single level (coarsest={coarsest})")
        self.coarse_inv, self.coarse_inv_host = dense_inverse_csr(self.ops[-1])
        # the dense kernel's column-major copy (None: the CSR form)
        self.coarse_dense = (torch.from_numpy(np.ascontiguousarray(self.coarse_inv_host.T)).to(dev)
                             if sell else None)
        # SELL-64 copies of the operators (level 0 too: the standalone solve's fine level) and transfers
        # (fine_sell=False: level 0's operator is the caller's own -- the Schur apply's matrix-free F / Gt_G)
        self.sells = [[sell_copy(M) if sell and (l > 0 or fine_sell or grp is not self.ops) else None
                       for l, M in enumerate(grp)] for grp in (self.ops, self.R, self.P)]
        # stencil-values copies of the large coarse levels (8 B per entry instead of 12 B; same bits)
        if svl_min_rows == "default":
            svl_min_rows = SVL_MIN_ROWS
        self.svls = [StencilValues.build(M, nf, self.sizes[l])
                     if (l > 0 and svl_min_rows is not None and M.shape[0] > svl_min_rows) else None
                     for l, M in enumerate(self.ops)]
        f64 = dict(dtype=torch.float64, device=dev)
        self.work = [[torch.zeros(M.shape[0], **f64) for _ in range(5)] for M in self.ops]
        self._levels = (_lib.MgLevel * len(self.ops))()
        empty_csr, empty_blk = _lib.Csr(0, 0, 0, None, None, None), _lib.RowBlocks(None, 0)
        for l, M in enumerate(self.ops):
            L = self._levels[l]
            L.nrows, L.pre, L.post = M.shape[0], pre, post
            L.lmin, L.lmax = self.bounds[l]
            L.A, L.A_blocks, L.diag = M.cstruct(), M.blocks.cstruct(), self.diags[l].data_ptr()
            if l < len(self.R):
                L.R, L.R_blocks = self.R[l].cstruct(), self.R[l].blocks.cstruct()
                L.P, L.P_blocks = self.P[l].cstruct(), self.P[l].blocks.cstruct()
            else:
                L.R = L.P = empty_csr
                L.R_blocks = L.P_blocks = empty_blk
            L.x, L.t, L.r, L.d, L.b = (w.data_ptr() for w in self.work[l])
            for name, grp in zip(("A_sell", "R_sell", "P_sell"), self.sells):
                S = grp[l] if l < len(grp) else None
                setattr(L, name, S.cstruct() if S is not None else _lib.Sell(0, 0, 0, 0, None, None, None, None))
            if self.svls[l] is not None:
                L.A_svl = ctypes.pointer(self.svls[l].cstruct())
        self._mg = _lib.Mg(len(self.ops), cycles, ctypes.cast(self._levels, ctypes.POINTER(_lib.MgLevel)),
                           self.coarse_inv.cstruct(), self.coarse_inv.blocks.cstruct(),
                           self.coarse_dense.data_ptr() if self.coarse_dense is not None else None)
        # the standalone solve's kernel choices (inside a Schur apply the preconditioner's own govern)
        self.kernel_opts = _lib.kernel_opts(kernel_opts)
        self._mg.opts = ctypes.pointer(self.kernel_opts)
        set_transfer_kinds(self._mg, self.fields, n)

    def set_matrix_free_transfers(self, on: bool):
        """Name (on) or hide (off) the field kinds in the hierarchy's struct: with them the whole-grid levels' transfers
        run matrix-free (same bits as the stored P / R)."""
        set_transfer_kinds(self._mg, self.fields if on else (), self.n)

    @property
    def nlevels(self) -> int:
        return len(self.ops)

    def cstruct(self) -> _lib.Mg:
        return self._mg

    def solve(self, b: torch.Tensor, out: torch.Tensor | None = None, sub: torch.Tensor | None = None) -> torch.Tensor:
        """x = MG^-1 b (``cycles`` V-cycles from 0); sub - x when sub is given."""
        n0 = self.ops[0].shape[0]
        assert b.is_cuda and b.dtype == torch.float64 and b.numel() == n0
        if out is None:
            out = torch.empty(n0, dtype=torch.float64, device=self.device)
        check(lib().mpbp_mg_solve(ctypes.byref(self._mg), ptr(b), ptr(sub), ptr(out), stream_handle()))
        return out

    def __repr__(self):
        return (f"Multigrid(levels={self.sizes}, fields={len(self.fields)}, pre={self.pre}, post={self.post}, "
                f"cycles={self.cycles}, ratio={self.ratio})")
