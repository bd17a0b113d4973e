"""Device-resident CSR matrices (HBM) driven through libmpbp's C ABI.

Layout in HBM: row_ptr int32[nrows+1], col_idx int32[nnz], val float64[nnz] -- the scipy.sparse
CSR layout, so a scipy matrix crosses the boundary with three copies and no reformatting.  Row
blocks (<= 256 rows, <= 4095 nonzeros each) are planned once on the host from row_ptr and kept
on the device; every SpMV-shaped kernel walks them.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_handle


class DeviceCSR:
    """A CSR matrix in HBM.  ``A @ x`` (x a CUDA float64 tensor) runs the HIP SpMV."""

    def __init__(self, row_ptr: torch.Tensor, col_idx: torch.Tensor, val: torch.Tensor, shape,
                 row_ptr_host: np.ndarray | None = None):
        assert row_ptr.dtype == torch.int32 and col_idx.dtype == torch.int32 and val.dtype == torch.float64
        assert row_ptr.is_cuda and col_idx.is_cuda and val.is_cuda
        self.row_ptr, self.col_idx, self.val = row_ptr, col_idx, val
        self.shape = (int(shape[0]), int(shape[1]))
        assert row_ptr.numel() == self.shape[0] + 1
        self._rp_host = row_ptr_host
        self._blocks = None
        self._cs = None
        self.stencil = None     # FStencil / PGStencil when the operator can be recomputed on the fly
        self.row_groups = 1     # rows = this many stacked fields over the same cells (plan_blocks order)

    # -- construction -------------------------------------------------------------------------
    @classmethod
    def from_scipy(cls, M, device=None):
        import scipy.sparse as sp
        M = sp.csr_matrix(M)
        M.sort_indices()
        dev = torch.device(device or "cuda")
        rp = np.ascontiguousarray(M.indptr, dtype=np.int32)
        return cls(torch.from_numpy(rp).to(dev),
                   torch.from_numpy(np.ascontiguousarray(M.indices, dtype=np.int32)).to(dev),
                   torch.from_numpy(np.ascontiguousarray(M.data, dtype=np.float64)).to(dev),
                   M.shape, row_ptr_host=rp)

    def to_scipy(self):
        import scipy.sparse as sp
        return sp.csr_matrix((self.val.cpu().numpy(), self.col_idx.cpu().numpy(), self.row_ptr.cpu().numpy()),
                             shape=self.shape)

    @property
    def nnz(self) -> int:
        return int(self.val.numel())

    @property
    def device(self):
        return self.val.device

    @property
    def row_ptr_host(self) -> np.ndarray:
        if self._rp_host is None:
            self._rp_host = self.row_ptr.cpu().numpy()
        return self._rp_host

    def cstruct(self) -> _lib.Csr:
        if self._cs is None:
            self._cs = _lib.Csr(self.shape[0], self.shape[1], self.nnz, self.row_ptr.data_ptr(),
                                self.col_idx.data_ptr(), self.val.data_ptr())
        return self._cs

    # -- row blocks -----------------------------------------------------------------------------
    def plan_blocks(self, row_begin=0, row_end=None, rows=None, groups=None):
        """Device row-block list over [row_begin, row_end), or over sorted row ranges `rows`.

        groups: the rows are `groups` equal stacked fields over the same cells (A: u_n, v_n, u_s, v_s, p;
        default self.row_groups).  The blocks are then listed cell-range-major across the fields, so the
        contiguous run of blocks each XCD takes (xcd_swizzle) covers the same cells of every field and the
        cross-field x gathers stay in that XCD's L2.  Order only: results are unchanged."""
        rp = self.row_ptr_host
        ranges = rows if rows is not None else [(row_begin, self.shape[0] if row_end is None else row_end)]
        pieces = []
        for a, b in ranges:
            need = lib().mpbp_plan_row_blocks(rp.ctypes.data_as(ctypes.c_void_p), a, b, None, 0)
            check(need)
            buf = np.empty(2 * max(int(need), 1), dtype=np.int32)
            lib().mpbp_plan_row_blocks(rp.ctypes.data_as(ctypes.c_void_p), a, b,
                                       buf.ctypes.data_as(ctypes.c_void_p), int(need))
            pieces.append(buf[: 2 * int(need)])
        pairs = np.concatenate(pieces) if pieces else np.zeros(0, dtype=np.int32)
        g = self.row_groups if groups is None else groups
        if g > 1 and rows is None and pairs.size and self.shape[0] % g == 0:
            gsize = self.shape[0] // g
            starts = pairs[0::2].astype(np.int64)
            gid = np.minimum(starts // gsize, g - 1)
            order = np.lexsort((gid, starts - gid * gsize))   # by position within the field, then field
            pairs = pairs.reshape(-1, 2)[order].reshape(-1)
        pairs = np.ascontiguousarray(pairs)
        blk = RowBlockList(torch.from_numpy(pairs).to(self.device), rp, pairs)
        blk.owner = self._identity()
        return blk

    def _identity(self):
        """What a row-block plan (its wave table in particular) was built from: this matrix's row structure."""
        return (self.row_ptr.data_ptr(), self.shape[0], self.nnz)

    @property
    def blocks(self):
        if self._blocks is None:
            self._blocks = self.plan_blocks()
        return self._blocks

    # -- kernels --------------------------------------------------------------------------------
    def matvec(self, x: torch.Tensor, out: torch.Tensor | None = None, mode=_lib.SPMV_STORE,
               z: torch.Tensor | None = None, blocks=None, order: str = "seq") -> torch.Tensor:
        """y = A x (or z + A x / z - A x by `mode`).  order "seq": each row summed left to right in CSR order
        (bit-identical to the oracle); "seg": a wavefront segmented reduction per row (mpbp_spmv_seg: within
        1e-12 of "seq", the north_star bar for apply.py:72's np.matmul)."""
        assert x.dtype == torch.float64 and x.is_cuda and x.numel() >= self.shape[1]
        if order not in ("seq", "seg"):
            raise ValueError(f"order must be 'seq' or 'seg', not {order!r}")
        if out is None:
            out = torch.empty(self.shape[0], dtype=torch.float64, device=self.device)
        bl = blocks or self.blocks
        # the wave table's fast path trusts row lengths read from the row_ptr the plan was made from: blocks planned
        # for another matrix (same shape, other pattern) would read wrong entries, so refuse them
        owner = getattr(bl, "owner", None)
        if owner is not None and owner != self._identity():
            raise ValueError("matvec: these row blocks were planned for another matrix (plan_blocks on this one)")
        blk = bl.cstruct()
        fn = lib().mpbp_spmv if order == "seq" else lib().mpbp_spmv_seg
        check(fn(ctypes.byref(self.cstruct()), ctypes.byref(blk), mode, ptr(x), ptr(z), ptr(out), stream_handle()))
        return out

    def __matmul__(self, other):
        if isinstance(other, DeviceCSR):
            return spgemm(self, other)
        if isinstance(other, np.ndarray) and other.ndim == 1:
            return self._host_matvec(other)
        if isinstance(other, np.ndarray):
            return self.matvec(torch.from_numpy(np.ascontiguousarray(other, dtype=np.float64))
                               .to(self.device)).cpu().numpy()
        return self.matvec(other)

    def _host_matvec(self, x: np.ndarray) -> np.ndarray:
        """A @ x for a host vector (apply.py:72 on host data; a host-side Krylov loop's operator): staged
        through page-locked buffers allocated on first use, so both PCIe copies run at DMA speed.  x must
        have exactly ncols entries (scipy's dimension check); one call at a time (a lock serialises threads)."""
        from .solve import _staged_host_call
        return _staged_host_call(self, x, self.shape[1], self.shape[0], self.device,
                                 lambda d_in, d_out: self.matvec(d_in, out=d_out))

    def release_staging(self):
        """Free the host-vector matvec's staging buffers (re-created on demand)."""
        self._pinned = None

    def diagonal(self, col_offset=0) -> torch.Tensor:
        d = torch.empty(self.shape[0], dtype=torch.float64, device=self.device)
        missing = ctypes.c_int32(0)
        check(lib().mpbp_csr_diag(ctypes.byref(self.cstruct()), col_offset, ptr(d), ctypes.byref(missing),
                                  stream_handle()))
        if missing.value:
            raise _lib.MpbpError(f"{missing.value} rows have no diagonal entry")
        return d

    def gershgorin(self, diag: torch.Tensor) -> float:
        out = ctypes.c_double(0.0)
        check(lib().mpbp_gershgorin(ctypes.byref(self.cstruct()), ptr(diag), ctypes.byref(out), stream_handle()))
        return out.value

    def extract(self, rows: torch.Tensor, colmap: torch.Tensor, ncols_local: int) -> "DeviceCSR":
        """Rows `rows` (global ids, device int32) with columns renumbered by `colmap` (device int32,
        global col -> local col or -1).  Entry order within a row is kept, so local row sums equal
        the global ones bit for bit.  Raises if a kept entry's column is unmapped."""
        nloc = rows.numel()
        row_nnz = torch.empty(max(nloc, 1), dtype=torch.int32, device=self.device)[:nloc]
        check(lib().mpbp_csr_extract_count(ctypes.byref(self.cstruct()), ptr(rows), nloc, ptr(row_nnz),
                                           stream_handle()))
        rp, ci, va = csr_from_row_nnz(row_nnz, (nloc, ncols_local), self.device)
        check(lib().mpbp_csr_extract_fill(ctypes.byref(self.cstruct()), ptr(rows), nloc, ptr(colmap), ptr(rp),
                                          ptr(ci), ptr(va), stream_handle()))
        return DeviceCSR(rp, ci, va, (nloc, ncols_local))

    def to_sell(self, ranges=None):
        """SELL-64 copy of the rows in `ranges` (list of [a, b) row ranges; default all rows)."""
        return DeviceSELL.from_csr(self, ranges)

    def __repr__(self):
        return f"DeviceCSR(shape={self.shape}, nnz={self.nnz}, device={self.device})"


class DeviceSELL:
    """SELL-64 copy of (some rows of) a DeviceCSR: one wavefront per 64-row slice, entries
    column-major in 16-byte pairs.  Row sums keep CSR order, so results equal the CSR kernels'."""

    def __init__(self, csr: DeviceCSR, slices: torch.Tensor, nslices: int, row_len, val, col, pair_rows: int):
        self.csr, self.slices, self.nslices = csr, slices, nslices
        self.row_len, self.val, self.col, self.pair_rows = row_len, val, col, pair_rows
        self.shape = csr.shape
        self._cs = _lib.Sell(csr.shape[0], csr.shape[1], nslices, 0,
                             slices.data_ptr() if nslices else None, row_len.data_ptr(),
                             val.data_ptr(), col.data_ptr())

    @classmethod
    def from_csr(cls, A: DeviceCSR, ranges=None):
        rp = A.row_ptr_host
        rg = np.asarray(ranges if ranges is not None else [(0, A.shape[0])], dtype=np.int32).reshape(-1, 2)
        rg = np.ascontiguousarray(rg)
        pr = ctypes.c_int64(0)
        need = check(lib().mpbp_sell_plan(rp.ctypes.data_as(ctypes.c_void_p), rg.ctypes.data_as(ctypes.c_void_p),
                                          rg.shape[0], None, 0, ctypes.byref(pr)))
        sl = np.zeros(4 * max(need, 1), dtype=np.int32)
        check(lib().mpbp_sell_plan(rp.ctypes.data_as(ctypes.c_void_p), rg.ctypes.data_as(ctypes.c_void_p),
                                   rg.shape[0], sl.ctypes.data_as(ctypes.c_void_p), need, ctypes.byref(pr)))
        dev = A.device
        slices = torch.from_numpy(sl).to(dev)
        row_len = torch.zeros(max(A.shape[0], 1), dtype=torch.uint8, device=dev)
        val = torch.zeros(max(pr.value, 1) * 128, dtype=torch.float64, device=dev)
        col = torch.zeros(max(pr.value, 1) * 128, dtype=torch.int32, device=dev)
        check(lib().mpbp_sell_fill(ctypes.byref(A.cstruct()), ptr(slices), int(need), ptr(row_len), ptr(val),
                                   ptr(col), stream_handle()))
        return cls(A, slices, int(need), row_len, val, col, int(pr.value))

    def sub(self, first: int, count: int):
        """The slices [first, first+count) as their own SELL view (shares storage)."""
        view = object.__new__(DeviceSELL)
        view.__dict__.update(self.__dict__)
        view.nslices = count
        view._cs = _lib.Sell(self.shape[0], self.shape[1], count, 0,
                             self.slices.data_ptr() + 16 * first if count else None, self.row_len.data_ptr(),
                             self.val.data_ptr(), self.col.data_ptr())
        return view

    def cstruct(self):
        return self._cs

    @property
    def device(self):
        return self.val.device

    def matvec(self, x, out=None, mode=_lib.SPMV_STORE, z=None):
        if out is None:
            out = torch.empty(self.shape[0], dtype=torch.float64, device=self.device)
        check(lib().mpbp_sell_spmv(ctypes.byref(self._cs), mode, ptr(x), ptr(z), ptr(out), stream_handle()))
        return out


class RowBlockList:
    """Row blocks of a CSR matrix in HBM (mpbp_rowblocks): the (start, end) pairs and, when the host row_ptr is given,
    the wave table (wave_table) the SpMV kernels start from."""

    def __init__(self, pairs: torch.Tensor, row_ptr_host: np.ndarray | None = None, pairs_host: np.ndarray | None = None):
        self.pairs = pairs
        self.count = pairs.numel() // 2
        self.table = None
        self.owner = None   # DeviceCSR._identity() of the matrix it was planned for (plan_blocks sets it)
        if row_ptr_host is not None and self.count:
            ph = pairs_host if pairs_host is not None else pairs.cpu().numpy()
            self.table = torch.from_numpy(wave_table(row_ptr_host, ph.reshape(-1, 2))).to(pairs.device)
        self._cs = _lib.RowBlocks(pairs.data_ptr() if self.count else None, self.count, 0,
                                  self.table.data_ptr() if self.table is not None else None)

    def cstruct(self):
        return self._cs


def wave_table(rp: np.ndarray, pairs: np.ndarray) -> np.ndarray:
    """Per row block 8 int32 (include/mpbp.h, mpbp_rowblocks.table): start row, end row, row_ptr at the starts of its
    four 64-row waves and at its end, and the waves' uniform-length flags (byte w = LEN in {8, 10, 12} when wave w's 64
    rows all hold LEN entries from an even offset)."""
    rp = np.asarray(rp, dtype=np.int64)
    ra, rb = pairs[:, 0].astype(np.int64), pairs[:, 1].astype(np.int64)
    t = np.zeros((pairs.shape[0], 8), dtype=np.int64)
    t[:, 0], t[:, 1] = ra, rb
    for w in range(5):
        t[:, 2 + w] = rp[np.minimum(ra + 64 * w, rb)]
    lens = np.diff(rp)
    flags = np.zeros(pairs.shape[0], dtype=np.int64)
    for w in range(4):
        a = ra + 64 * w
        full = rb - a >= 64
        idx = np.nonzero(full)[0]
        if idx.size:
            rows = a[idx][:, None] + np.arange(64)[None, :]
            L = lens[rows]
            L0 = L[:, 0]
            ok = np.all(L == L0[:, None], axis=1) & np.isin(L0, (8, 10, 12)) & (rp[a[idx]] % 2 == 0)
            flags[idx] |= np.where(ok, L0, 0) << (8 * w)
    t[:, 7] = flags
    return t.astype(np.int32).reshape(-1)


def csr_from_row_nnz(row_nnz: torch.Tensor, shape, device):
    """Allocate row_ptr/col_idx/val for the given per-row counts (device exclusive scan)."""
    rows = row_nnz.numel()
    row_ptr = torch.empty(rows + 1, dtype=torch.int32, device=device)
    total = ctypes.c_int64(0)
    check(lib().mpbp_exclusive_scan(ptr(row_nnz), ptr(row_ptr), rows, ctypes.byref(total), stream_handle()))
    col = torch.empty(max(total.value, 1), dtype=torch.int32, device=device)[: total.value]
    val = torch.empty(max(total.value, 1), dtype=torch.float64, device=device)[: total.value]
    return row_ptr, col, val


def spgemm(A: DeviceCSR, B: DeviceCSR, alpha: float = 1.0) -> DeviceCSR:
    """alpha * A @ B keeping every structural product (solve.py:246-249 use np.matmul)."""
    if A.shape[1] != B.shape[0]:
        raise ValueError(f"shape mismatch {A.shape} @ {B.shape}")
    row_nnz = torch.empty(A.shape[0], dtype=torch.int32, device=A.device)
    check(lib().mpbp_spgemm_count(ctypes.byref(A.cstruct()), ctypes.byref(B.cstruct()), ptr(row_nnz),
                                  stream_handle()))
    rp, ci, va = csr_from_row_nnz(row_nnz, (A.shape[0], B.shape[1]), A.device)
    check(lib().mpbp_spgemm_fill(ctypes.byref(A.cstruct()), ctypes.byref(B.cstruct()), float(alpha), ptr(rp),
                                 ptr(ci), ptr(va), stream_handle()))
    return DeviceCSR(rp, ci, va, (A.shape[0], B.shape[1]))
