"""Row partition of the MAC grid over ranks (one process per GPU) with halo exchange over RCCL.

Every field (u_n, v_n, u_s, v_s, p) is an n x n grid stored row-major; rank k owns grid rows
[r0, r1) of every field.  A rank's vector is laid out "owned first, then ghosts":

    owned:  field-major, f * L*n + (gr - r0)*n + c                  (L = r1 - r0)
    ghosts: h rows above (r0-h .. r0-1) of every field, then h rows below (r1 .. r1+h-1) of every
            field (periodic): above row j of field f at (f*h + j)*n, below at (nf*h + f*h + j)*n

Matrices keep their global row order inside a rank and have their columns renumbered into that
layout (``DeviceCSR.extract``), so every local row sum is the global one, bit for bit.  Before a
sweep reads a vector its ghost rows are refreshed while the rows that touch no ghost (the interior)
are computed; the boundary rows run after.  Two exchange implementations:

* ``RcclHalo`` (default with the nccl = RCCL backend): libmpbp's own RCCL communicator; the exchange is
  issued from C inside ``mpbp_schur_apply`` (no Python between the kernels): a four-field vector's
  boundary rows are packed by one gather kernel, then one RCCL group of neighbour ncclSend / ncclRecv
  writes straight into the ghost rows, in order on the apply stream (``MPBP_HALO_IN_ORDER``, default; a
  side-stream variant forked / joined by events is ``halo_overlap=True``).  With the communication-
  avoiding schedule (``ca``) an apply makes two such exchanges.
* ``HaloExchanger`` (gloo, CPU-staged; the tests' backend): packs the top/bottom h owned rows of every
  field, all-gathers them, copies the neighbours' strips into the ghost slots.

The halo depth h of each vector kind is measured from the matrices that read it (F, D read
velocity: h = 1; G, Gt_G, Gt_F_G read pressure: h = 2 for Gt_F_G).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_handle
from .csr import DeviceCSR, spgemm
from .preconditioner import PGStencil
from .solve import PlanProfiling, _capture, _pg_stencil

N_VEL_FIELDS = 4
N_P_FIELDS = 1


@dataclass
class RowPartition:
    n: int
    world: int
    rank: int
    ghosts: bool = False   # ghost slots even at world = 1 (the periodic self-exchange; tests the halo path)
    bounds: tuple | None = None   # explicit ((r0, rows) per rank); default: n split evenly (the first n % world +1)
    allow_empty: bool = False     # coarse multigrid levels (level_partitions) may leave a rank without rows

    def __post_init__(self):
        self.ghosts = self.ghosts or self.world > 1
        if self.bounds is None:
            base, rem = divmod(self.n, self.world)
            self.bounds = tuple((k * base + min(k, rem), base + (1 if k < rem else 0)) for k in range(self.world))
        self.bounds = tuple((int(a), int(b)) for a, b in self.bounds)
        if len(self.bounds) != self.world or sum(b for _, b in self.bounds) != self.n:
            raise ValueError(f"row bounds {self.bounds} do not cover the {self.n} grid rows once")
        start = 0   # contiguous, in rank order, every rank at least one row (the halo and gather layouts assume it)
        for k, (a, b) in enumerate(self.bounds):
            if a != start or b < (0 if self.allow_empty else 1):
                raise ValueError(f"row bounds {self.bounds}: rank {k} must start at row {start} and own "
                                 f"{'>= 0 rows' if self.allow_empty else '>= 1 row'}")
            start += b
        self.r0, self.L = self.bounds[self.rank]
        self.r1 = self.r0 + self.L
        self.min_rows = min(b for _, b in self.bounds)

    def coarse(self, levels: int = 1) -> "RowPartition | None":
        """The same ranks' rows of the grid coarsened `levels` times by 2 (rows [r0 / 2^l, r1 / 2^l)), or None when
        some rank's rows do not halve exactly."""
        f = 1 << levels
        if self.n % f or any(a % f or b % f for a, b in self.bounds):
            return None
        return RowPartition(self.n // f, self.world, self.rank, self.ghosts, tuple((a // f, b // f) for a, b in self.bounds),
                            allow_empty=True)

    @property
    def N(self):
        return self.n * self.n

    def n_owned(self, nfields):
        return nfields * self.L * self.n

    def n_ext(self, nfields, h):
        return self.n_owned(nfields) + (nfields * 2 * h * self.n if self.ghosts else 0)

    def owned_rows(self, nfields) -> np.ndarray:
        """Global ids (in a field-major vector of nfields fields) of the owned unknowns, local order."""
        n, N = self.n, self.N
        return np.concatenate([f * N + np.arange(self.r0 * n, self.r1 * n, dtype=np.int64) for f in range(nfields)])

    def ext_rows(self, nfields, h) -> np.ndarray:
        """Global id of every slot of the owned + ghost ("ext") layout: owned rows field-major, then h rows
        above of every field (increasing row order), then h rows below of every field (periodic)."""
        n, N = self.n, self.N
        cols = np.arange(n, dtype=np.int64)
        above = [f * N + ((self.r0 - h + j) % n) * n + cols for f in range(nfields) for j in range(h)]
        below = [f * N + ((self.r1 + j) % n) * n + cols for f in range(nfields) for j in range(h)]
        parts = [self.owned_rows(nfields)] + (above + below if self.ghosts else [])
        return np.concatenate(parts)

    def colmap(self, nfields, h) -> np.ndarray:
        """Global column -> local ext index (-1 where the rank holds no copy)."""
        n, N, L = self.n, self.N, self.L
        cm = np.full(nfields * N, -1, dtype=np.int32)
        own = self.n_owned(nfields)
        if self.world > 1:
            if self.min_rows < h:
                raise ValueError(f"halo depth {h} exceeds the {self.min_rows} grid rows of the smallest rank")
            cols = np.arange(n, dtype=np.int64)
            for f in range(nfields):
                for j in range(h):
                    top = (self.r0 - h + j) % n
                    bot = (self.r1 + j) % n
                    cm[f * N + top * n + cols] = own + (f * h + j) * n + cols
                    cm[f * N + bot * n + cols] = own + (nfields * h + f * h + j) * n + cols
        for f in range(nfields):
            cm[f * N + self.r0 * n: f * N + self.r1 * n] = f * L * n + np.arange(L * n, dtype=np.int32)
        return cm


def _row_diagonal(M, row_gid: torch.Tensor) -> torch.Tensor:
    """Diagonal of a row subset of an operator with global columns (row i of M is global row row_gid[i])."""
    counts = (M.row_ptr[1:] - M.row_ptr[:-1]).to(torch.int64)
    owner = torch.repeat_interleave(torch.arange(M.shape[0], device=M.col_idx.device), counts)
    hit = M.col_idx.to(torch.int64) == row_gid.to(torch.int64)[owner]
    d = torch.zeros(M.shape[0], dtype=torch.float64, device=M.val.device)
    d[owner[hit]] = M.val[hit]
    if int(hit.sum()) != M.shape[0]:
        raise _lib.MpbpError("rank-local product: a row has no diagonal entry")
    return d


def _gtg_stencil(D, G):
    """The matrix-free Gt_G policy of the global product (commutator_products), for a rank-local product."""
    sd, sg = getattr(D, "stencil", None), getattr(G, "stencil", None)
    if isinstance(sd, PGStencil) and sd.op == _lib.PG_D and isinstance(sg, PGStencil) and sg.op == _lib.PG_G \
            and sd.same_grid(sg):
        return PGStencil(sd.prm, sd.cell, _lib.PG_GTG)
    return None


def halo_reach(row_ptr: torch.Tensor, col_idx: torch.Tensor, row_gid: torch.Tensor, n: int) -> int:
    """Largest periodic grid-row distance between a row and the columns it reads."""
    N = n * n
    counts = (row_ptr[1:] - row_ptr[:-1]).to(torch.int64)
    if col_idx.numel() == 0:
        return 0
    rgr = torch.repeat_interleave((row_gid.to(torch.int64) % N) // n, counts)
    cgr = (col_idx.to(torch.int64) % N) // n
    d = torch.remainder(cgr - rgr, n)
    return int(torch.minimum(d, n - d).max().item())


def ghost_depth(col_idx: torch.Tensor, n: int, r0: int, L: int) -> int:
    """Deepest ghost row the columns `col_idx` (global ids of stacked n x n fields) reach outside the owned grid
    rows [r0, r0 + L), periodic; 0 when every column is owned."""
    if col_idx.numel() == 0:
        return 0
    gr = (col_idx.to(torch.int64) % (n * n)) // n
    above = torch.remainder(r0 - gr, n)          # rows above r0 (1 = the row just above)
    below = torch.remainder(gr - (r0 + L - 1), n)   # rows below the last owned row
    inside = torch.remainder(gr - r0, n) < L
    d = torch.where(inside, torch.zeros_like(gr), torch.minimum(above, below))
    return int(d.max().item())


def boundary_ranges(row_ptr: torch.Tensor, col_idx: torch.Tensor, n_owned_cols: int):
    """(interior, boundary) lists of [a, b) row ranges: a boundary row reads a ghost column."""
    nrows = row_ptr.numel() - 1
    counts = (row_ptr[1:] - row_ptr[:-1]).to(torch.int64)
    rows = torch.repeat_interleave(torch.arange(nrows, device=col_idx.device), counts)
    flag = torch.zeros(nrows, dtype=torch.bool, device=col_idx.device)
    flag[rows[col_idx.to(torch.int64) >= n_owned_cols]] = True
    f = flag.cpu().numpy().astype(np.int8)
    edges = np.flatnonzero(np.diff(np.concatenate([[-1], f, [-1]])) != 0)
    inner, bnd = [], []
    for a, b in zip(edges[:-1], edges[1:]):
        (bnd if f[a] else inner).append((int(a), int(b)))
    return inner, bnd


class HaloExchanger:
    """All-gather of every rank's top/bottom h owned rows per field; ghosts filled from neighbours."""

    def __init__(self, part: RowPartition, nfields: int, h: int, device, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.part, self.nf, self.h, self.group = part, nfields, h, group
        self.hn = h * part.n
        self.device = torch.device(device)
        backend = dist.get_backend(group)
        self.stage_cpu = backend != "nccl" and self.device.type != "cpu"
        bdev = torch.device("cpu") if self.stage_cpu else self.device
        self.send = torch.empty(nfields * 2 * self.hn, dtype=torch.float64, device=bdev)
        self.recv = torch.empty(part.world * nfields * 2 * self.hn, dtype=torch.float64, device=bdev)
        self.use_base = backend == "nccl"
        self.work = None

    def _pack(self, x_ext):
        own = x_ext[: self.part.n_owned(self.nf)].view(self.nf, self.part.L * self.part.n)
        s = (torch.empty(self.nf, 2, self.hn, dtype=torch.float64, device=x_ext.device)
             if self.stage_cpu else self.send.view(self.nf, 2, self.hn))
        s[:, 0] = own[:, : self.hn]
        s[:, 1] = own[:, own.shape[1] - self.hn:]
        if self.stage_cpu:
            self.send.copy_(s.reshape(-1))

    def begin(self, x_ext: torch.Tensor):
        self._pack(x_ext)
        if self.use_base:
            self.work = self.dist.all_gather_into_tensor(self.recv, self.send, group=self.group, async_op=True)
        else:
            chunks = list(self.recv.view(self.part.world, -1).unbind(0))
            self.work = self.dist.all_gather(chunks, self.send, group=self.group, async_op=True)

    def end(self, x_ext: torch.Tensor):
        if self.work is not None:
            self.work.wait()
            self.work = None
        k, W = self.part.rank, self.part.world
        R = self.recv.view(W, self.nf, 2, self.hn)
        g = x_ext[self.part.n_owned(self.nf): self.part.n_ext(self.nf, self.h)].view(2, self.nf, self.hn)
        g[0] = R[(k - 1) % W, :, 1].to(g.device, non_blocking=True)     # rows above: up's bottom rows
        g[1] = R[(k + 1) % W, :, 0].to(g.device, non_blocking=True)     # rows below: down's top rows

    def exchange(self, x_ext):
        self.begin(x_ext)
        self.end(x_ext)


class Gatherer:
    """All-gather of a row-partitioned nf-field vector into the whole field-major vector (gloo / host-staged; the
    RCCL form is mpbp_halo_allgather): rank k owns rows [r0_k, r0_k + L_k) of every field of an n x n grid."""

    def __init__(self, nf: int, n: int, bounds, rank: int, group=None):
        import torch.distributed as dist
        self.dist, self.group, self.nf, self.n, self.rank = dist, group, nf, n, rank
        self.bounds = tuple(bounds)
        self.lmax = max(b for _, b in self.bounds)
        per = nf * self.lmax * n
        self.send = torch.zeros(per, dtype=torch.float64)
        self.recv = torch.zeros(len(self.bounds) * per, dtype=torch.float64)
        idx = np.empty(nf * n * n, dtype=np.int64)
        for k, (r0, L) in enumerate(self.bounds):
            for f in range(nf):
                idx[f * n * n + r0 * n: f * n * n + (r0 + L) * n] = k * per + f * self.lmax * n + np.arange(L * n)
        self.idx = torch.from_numpy(idx)

    def gather(self, x_owned: torch.Tensor, x_full: torch.Tensor):
        L = self.bounds[self.rank][1]
        own = x_owned[: self.nf * L * self.n].view(self.nf, L * self.n).cpu()
        self.send.view(self.nf, self.lmax * self.n)[:, : L * self.n] = own
        chunks = list(self.recv.view(len(self.bounds), -1).unbind(0))
        self.dist.all_gather(chunks, self.send, group=self.group)
        x_full[: self.idx.numel()] = self.recv[self.idx].to(x_full.device)


def rccl_library_path() -> str:
    """The RCCL torch itself loaded (one RCCL per process), else ROCm's."""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "/opt/rocm/lib/librccl.so"


class RcclHalo:
    """Ghost-row exchange in libmpbp (csrc/halo.cpp): one gather kernel packs a four-field vector's
    boundary rows (before the group opens), then one RCCL group of neighbour sends / receives writes the
    ghost rows; issued from C inside mpbp_schur_apply -- no Python callback, no all-gather.
    The communicator is libmpbp's own (its unique id travels over `group`); world = 1 exchanges with
    itself (the periodic wrap)."""

    # one RCCL communicator per process group: the first RcclHalo of a group opens it (collective), later ones -- the
    # partitioned preconditioners and their multigrid levels -- share it (mpbp_halo_create_shared, local), so a rank
    # holds one communicator however many preconditioners it builds.  The key is the group's global ranks (stable, unlike
    # id(group)), and whether to share is agreed over the group (an all-reduce MIN of "this rank has a live one"): if
    # any rank lacks it, every rank opens a new communicator together, so no rank waits in a collective the others skip.
    _by_group: dict = {}

    @staticmethod
    def _group_key(part: RowPartition, group):
        import torch.distributed as dist
        g = group if group is not None else dist.group.WORLD
        return (tuple(dist.get_process_group_ranks(g)), part.world, part.rank)

    @staticmethod
    def _agree(have: bool, part: RowPartition, group) -> bool:
        if part.world == 1:
            return have
        import torch.distributed as dist
        dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
        t = torch.tensor([1 if have else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        return bool(t.item())

    def __init__(self, part: RowPartition, h_u: int, h_p: int, group=None, overlap: bool = False, share: bool = True):
        """share=False opens a communicator of this object's own (collective over `group`, every rank must pass the same
        value); share=True attaches to the group's existing one when every rank still holds it."""
        import weakref
        key = self._group_key(part, group) if share else None
        ref = RcclHalo._by_group.get(key) if share else None
        base = ref() if ref is not None else None
        have = base is not None and bool(base.handle)
        if share and self._agree(have, part, group):
            self.handle = ctypes.c_void_p()
            check(lib().mpbp_halo_create_shared(base.handle, part.n, part.r0, part.L, h_u, h_p,
                                                ctypes.byref(self.handle)))
            self._finish(overlap)
            return
        path = rccl_library_path().encode()
        uid = (ctypes.c_uint8 * 128)()
        if part.world == 1:
            check(lib().mpbp_rccl_unique_id(path, uid))
        else:
            import torch.distributed as dist
            box = [None]
            if part.rank == 0:
                check(lib().mpbp_rccl_unique_id(path, uid))
                box = [bytes(uid)]
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                       group=group)
            ctypes.memmove(uid, box[0], 128)
        self.handle = ctypes.c_void_p()
        check(lib().mpbp_halo_create(path, uid, part.world, part.rank, part.n, part.r0, part.L, h_u, h_p,
                                     ctypes.byref(self.handle)))
        if share:
            RcclHalo._by_group[key] = weakref.ref(self)
        self._finish(overlap)

    @property
    def comm(self) -> int:
        """Identity of the RCCL communicator this object exchanges over (mpbp_halo_comm)."""
        return int(lib().mpbp_halo_comm(self.handle) or 0)

    @property
    def comm_refs(self) -> int:
        """Halo objects of this process holding the same communicator."""
        return int(lib().mpbp_halo_comm_refs(self.handle))

    def _finish(self, overlap):
        check(lib().mpbp_halo_set_mode(self.handle, _lib.HALO_OVERLAP if overlap else _lib.HALO_IN_ORDER))
        self.overlap = overlap
        self.fn = _lib.HALO_FN(ctypes.cast(lib().mpbp_halo_exchange, ctypes.c_void_p).value)
        self.pair_fn = _lib.HALO_PAIR_FN(ctypes.cast(lib().mpbp_halo_exchange_pair, ctypes.c_void_p).value)
        self.gather_fn = _lib.GATHER_FN(ctypes.cast(lib().mpbp_halo_allgather, ctypes.c_void_p).value)

    def add_kind(self, part: RowPartition, nfields: int, h: int, overlap: bool | None = None) -> int:
        """Another vector layout on this communicator (mpbp_halo_add_kind); returns its kind id."""
        ov = self.overlap if overlap is None else overlap
        return check(lib().mpbp_halo_add_kind(self.handle, nfields, part.n, part.r0, part.L, h,
                                              _lib.HALO_OVERLAP if ov else _lib.HALO_IN_ORDER))

    def add_gather(self, nfields: int, n: int, bounds) -> int:
        """An all-gather layout (mpbp_halo_add_gather): bounds = ((r0, rows) per rank)."""
        r0s = np.ascontiguousarray([a for a, _ in bounds], dtype=np.int32)
        rows = np.ascontiguousarray([b for _, b in bounds], dtype=np.int32)
        return check(lib().mpbp_halo_add_gather(self.handle, nfields, n, r0s.ctypes.data_as(ctypes.c_void_p),
                                                rows.ctypes.data_as(ctypes.c_void_p)))

    def check(self):
        if lib().mpbp_halo_status(self.handle) != 0:
            raise _lib.MpbpError(lib().mpbp_halo_last_error(self.handle).decode())

    def close(self):
        if self.handle:
            lib().mpbp_halo_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _Halos:
    """The ghost-row exchanges and all-gathers of one partitioned object: RCCL (libmpbp's halo object; the callbacks
    are its C functions) or torch / gloo (host-staged; Python callbacks looked up by vector address)."""

    def __init__(self, impl: str, rccl: "RcclHalo | None", group, device):
        self.impl, self.rccl, self.group, self.device = impl, rccl, group, torch.device(device)
        self._ex, self._gather, self._tensors = {}, {}, {}
        if rccl is not None:
            self.fn, self.gather_fn, self.ctx = rccl.fn, rccl.gather_fn, rccl.handle
        else:
            self.fn = _lib.HALO_FN(self._halo)
            self.gather_fn = _lib.GATHER_FN(self._allgather)
            self.ctx = None

    def add_kind(self, part: RowPartition, nfields: int, h: int, kind: int | None = None) -> int:
        if self.rccl is not None:
            return self.rccl.add_kind(part, nfields, h) if kind is None else kind
        k = len(self._ex) if kind is None else kind
        while kind is None and k in self._ex:
            k += 1
        self._ex[k] = HaloExchanger(part, nfields, h, self.device, self.group)
        return k

    def add_gather(self, nfields: int, n: int, bounds, rank: int) -> int:
        if self.rccl is not None:
            return self.rccl.add_gather(nfields, n, bounds)
        g = len(self._gather)
        self._gather[g] = Gatherer(nfields, n, bounds, rank, self.group)
        return g

    def register(self, *tensors):
        for t in tensors:
            self._tensors[t.data_ptr()] = t

    # ctypes prints and swallows an exception raised inside a callback, and the C apply would go on with stale ghost
    # rows: the callbacks record the first failure instead, and check() raises it once the apply has returned (as
    # RcclHalo.check does with mpbp_halo_status)
    error = None

    def _halo(self, ctx, kind, x_ptr, phase, stream):
        if self.error is not None:
            return
        try:
            x = self._tensors[int(x_ptr)]
            ex = self._ex[int(kind)]
            if phase == _lib.HALO_BEGIN:
                ex.begin(x)
            else:
                ex.end(x)
        except BaseException as e:   # noqa: BLE001 -- re-raised by check()
            self.error = e

    def _allgather(self, ctx, gid, own_ptr, full_ptr, stream):
        if self.error is not None:
            return
        try:
            self._gather[int(gid)].gather(self._tensors[int(own_ptr)], self._tensors[int(full_ptr)])
        except BaseException as e:   # noqa: BLE001
            self.error = e

    def check(self):
        """Raise the first exception a host-staged exchange or gather hit during the last apply."""
        if self.rccl is not None:
            self.rccl.check()
        if self.error is not None:
            e, self.error = self.error, None
            raise RuntimeError(f"halo exchange failed inside the apply: {type(e).__name__}: {e}") from e


def level_partitions(part: RowPartition, sizes) -> list[RowPartition]:
    """The row partition of every multigrid level: level l + 1's rows of a rank are [ceil(r0 / 2), ceil(r1 / 2)) of its
    level-l rows [r0, r1) -- exact halving for even bounds, a disjoint cover of the coarse grid in any case."""
    parts = [part]
    for m in sizes[1:]:
        p = parts[-1]
        b = tuple(((a + 1) // 2, (a + L + 1) // 2 - (a + 1) // 2) for a, L in p.bounds)
        parts.append(RowPartition(m, part.world, part.rank, part.ghosts, b, allow_empty=True))
    return parts


def _csr_rows(M: DeviceCSR, idx: torch.Tensor) -> DeviceCSR:
    """Rows idx (local row numbers of M, device) of M in that order: entries and their order kept, columns as they are."""
    rp = M.row_ptr.to(torch.int64)
    idx = idx.to(torch.int64)
    lens = rp[idx + 1] - rp[idx]
    nrp = torch.zeros(idx.numel() + 1, dtype=torch.int64, device=rp.device)
    torch.cumsum(lens, 0, out=nrp[1:])
    owner = torch.repeat_interleave(torch.arange(idx.numel(), device=rp.device), lens)
    src = rp[idx][owner] + (torch.arange(int(nrp[-1]), device=rp.device) - nrp[:-1][owner])
    return DeviceCSR(nrp.to(torch.int32), M.col_idx[src].contiguous(), M.val[src].contiguous(), (idx.numel(), M.shape[1]))


def _positions(keys: torch.Tensor, v: torch.Tensor, bad: torch.Tensor | None = None) -> torch.Tensor:
    """Positions of the values v in the sorted `keys` (every value must be a key).  bad (a device bool, optional):
    OR-ed with "some value is not a key" and left for the caller to check once (no device synchronisation here);
    without it the check is made at once."""
    k = keys.to(torch.int64)
    vv = v.to(torch.int64)
    pos = torch.searchsorted(k, vv)
    if v.numel():
        miss = (pos >= k.numel()) | (k[pos.clamp(max=max(k.numel() - 1, 0))] != vv)
        if bad is not None:
            bad |= miss.any()
        elif bool(miss.any()):
            raise ValueError("a row / column outside this rank's band")
    return pos


def _relabel_cols(M: DeviceCSR, keys: torch.Tensor, bad: torch.Tensor | None = None) -> DeviceCSR:
    """M with every column replaced by its position in the sorted `keys`: the same entries in the same order (the
    relabelling is monotone), as a product's left operand indexing the rows `keys` of the right one."""
    return DeviceCSR(M.row_ptr, _positions(keys, M.col_idx, bad).to(torch.int32), M.val, (M.shape[0], keys.numel()))


def _allgather_csr(M: DeviceCSR, rows: torch.Tensor, nrows: int, group) -> DeviceCSR:
    """The whole operator from every rank's rows: M holds the global rows `rows` of this rank (global columns); the
    result has every one of the `nrows` rows in global order, each row's entries in their order."""
    import torch.distributed as dist
    dev = M.val.device
    cdev = dev if dist.get_backend(group) == "nccl" else torch.device("cpu")
    world = dist.get_world_size(group)
    lens = (M.row_ptr[1:] - M.row_ptr[:-1]).to(torch.int64)
    meta = torch.tensor([rows.numel(), M.col_idx.numel()], dtype=torch.int64, device=cdev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    cnt = [(int(m[0]), int(m[1])) for m in metas]

    def gather(t, k, dtype):
        size = max(max(c[k] for c in cnt), 1)
        buf = torch.zeros(size, dtype=dtype, device=cdev)
        buf[: t.numel()] = t.to(device=cdev, dtype=dtype)
        outs = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(outs, buf, group=group)
        return torch.cat([o[: c[k]] for o, c in zip(outs, cnt)]).to(dev)
    r_all, l_all = gather(rows, 0, torch.int64), gather(lens, 0, torch.int64)
    c_all, v_all = gather(M.col_idx, 1, torch.int64), gather(M.val, 1, torch.float64)
    perm = torch.argsort(r_all)
    if r_all.numel() != nrows or not bool((r_all[perm] == torch.arange(nrows, device=dev)).all()):
        raise ValueError("the ranks' rows do not cover the level exactly once")
    start = torch.zeros(nrows + 1, dtype=torch.int64, device=dev)
    torch.cumsum(l_all, 0, out=start[1:])
    ls = l_all[perm]
    rp = torch.zeros(nrows + 1, dtype=torch.int64, device=dev)
    torch.cumsum(ls, 0, out=rp[1:])
    owner = torch.repeat_interleave(torch.arange(nrows, device=dev), ls)
    src = start[perm][owner] + (torch.arange(int(rp[-1]), device=dev) - rp[:-1][owner])
    return DeviceCSR(rp.to(torch.int32), c_all[src].to(torch.int32).contiguous(), v_all[src].contiguous(),
                     (nrows, M.shape[1]))


def mg_part_cap(sizes, part: RowPartition, nfields: int, min_cells: int = 1 << 14,
                max_part_levels: int | None = None) -> int:
    """The levels [0, cap) a row-partitioned hierarchy may split by size alone: PartitionedMultigrid's rule without
    the ghost-depth test (which can only stop it earlier)."""
    nl = len(sizes)
    parts = level_partitions(part, sizes)
    cap = nl - 1 if max_part_levels is None else max(1, min(nl - 1, max_part_levels))
    for l in range(1, nl - 1):
        q = parts[l]
        if l >= cap or nfields * q.n * q.n // part.world < min_cells or q.min_rows < 1:
            return l
    return nl - 1


def mg_bands(sizes, fields, part: RowPartition, cap: int, device) -> list:
    """S_l, l = 0 .. cap: the rows of level l (sorted global ids, device int32) a rank forms to have its owned rows of
    every level down to `cap`: S_cap = the owned rows, S_l = the owned rows and every fine row the restriction of
    S_{l+1} reads (A_{l+1} = R_l (A_l P_l) row by row needs exactly those rows of A_l)."""
    from .mg import transfer_rows
    nf = len(fields)
    parts = level_partitions(part, sizes)
    own = [torch.from_numpy(q.owned_rows(nf).astype(np.int32)).to(device) for q in parts[: cap + 1]]
    S = [None] * (cap + 1)
    S[cap] = own[cap]
    for l in range(cap - 1, -1, -1):
        R = transfer_rows(sizes[l], fields, _lib.MG_R, S[l + 1])
        S[l] = torch.unique(torch.cat([own[l], R.col_idx])).to(torch.int32)
    return S


class LocalHierarchy:
    """The multigrid levels one rank of a row partition needs, formed from its own rows: no global operator on any
    rank (setup memory O(N / world + ghosts) down to the replicated coarse levels).

    A0 holds the rows S[0] (mg_bands) of level 0's operator with their global columns (assembled, or the rank-local
    product rows of Gt_G).  Level l + 1's band is R_l[S_{l+1}] (A_l[S_l] P_l) with the restriction's columns relabelled
    into S_l and A_l's into the fine rows it reaches (monotone relabellings: each product row performs the global
    SpGEMM's operations in its order -- the one-GPU hierarchy's rows bit for bit), the transfers' rows built for those
    rows only (mpbp_mg_transfer_rows_*).  replicated(P) all-gathers the ranks' owned rows of level P and coarsens
    that level as mg.Multigrid does (the levels below are small): the same operators as the one-GPU hierarchy's."""

    def __init__(self, A0: DeviceCSR, S: list, sizes, fields, part: RowPartition, group=None, pre=2, post=2,
                 cycles=1, ratio=4.0, coarsest=8, stamp=None):
        from .mg import transfer_rows
        stamp = stamp or (lambda name: None)
        self.device = A0.val.device
        self.sizes, self.fields, self.n, self.nf = list(sizes), tuple(fields), int(sizes[0]), len(fields)
        self.nlevels = len(self.sizes)
        self.pre, self.post, self.cycles, self.ratio, self.coarsest = pre, post, cycles, ratio, coarsest
        self.S, self.part, self.group = S, part, group
        if A0.shape[0] != S[0].numel():
            raise ValueError("A0 must hold the band rows S[0]")
        self.band = [A0]
        bad = torch.zeros((), dtype=torch.bool, device=self.device)   # checked once (each sync costs under contention)
        for l in range(len(S) - 1):
            A = self.band[l]
            C = torch.unique(A.col_idx)
            AP = spgemm(_relabel_cols(A, C, bad), transfer_rows(self.sizes[l], self.fields, _lib.MG_P, C))
            R = transfer_rows(self.sizes[l], self.fields, _lib.MG_R, S[l + 1])
            self.band.append(spgemm(_relabel_cols(R, S[l], bad), AP))
            del AP, R
            stamp(f"mg_band_level{l + 1}")
        if bool(bad):
            raise ValueError("LocalHierarchy: a restriction row reads outside its band (mg_bands)")
        self._rep = {}
        self.stamp = stamp

    def op_rows(self, l: int, rows: torch.Tensor) -> DeviceCSR:
        return _csr_rows(self.band[l], _positions(self.S[l], rows))

    def R_rows(self, l: int, rows: torch.Tensor) -> DeviceCSR:
        from .mg import transfer_rows
        return transfer_rows(self.sizes[l], self.fields, _lib.MG_R, rows)

    def P_rows(self, l: int, rows: torch.Tensor) -> DeviceCSR:
        from .mg import transfer_rows
        return transfer_rows(self.sizes[l], self.fields, _lib.MG_P, rows)

    def diag_rows(self, l: int, rows: torch.Tensor) -> torch.Tensor:
        return _row_diagonal(self.op_rows(l, rows), rows)

    def bounds(self, l: int, rows: torch.Tensor):
        """(lmin, lmax) of level l's smoother: the Gershgorin bound is the maximum over the ranks of their owned rows'
        (every row's sum is the global operator's): the one-GPU hierarchy's bound, exactly."""
        import torch.distributed as dist
        lm = self.op_rows(l, rows).gershgorin(self.diag_rows(l, rows)) if rows.numel() else 0.0
        cdev = self.device if dist.get_backend(self.group) == "nccl" else "cpu"
        t = torch.tensor([lm], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        lmax = float(t.item())
        return lmax / self.ratio, lmax

    def replicated(self, P: int):
        """mg.Multigrid of level P's whole operator (every rank's owned rows of it, all-gathered): levels P .. end."""
        if P not in self._rep:
            from .mg import Multigrid
            q = level_partitions(self.part, self.sizes)[P]
            own = torch.from_numpy(q.owned_rows(self.nf).astype(np.int32)).to(self.device)
            full = _allgather_csr(self.op_rows(P, own), own, self.nf * self.sizes[P] ** 2, self.group)
            self.stamp("mg_gather_level")
            if P == self.nlevels - 1:   # only the coarsest level: its dense inverse
                self._rep[P] = _CoarsestLevel(full, self.ratio)
            else:
                sub = Multigrid(full, self.sizes[P], self.fields, pre=self.pre, post=self.post, cycles=self.cycles,
                                ratio=self.ratio, coarsest=self.coarsest, fine_sell=True)
                if sub.sizes != self.sizes[P:]:
                    raise AssertionError(f"coarse levels {sub.sizes} != {self.sizes[P:]}")
                self._rep[P] = sub
            self.stamp("mg_replicated_levels")
        return self._rep[P]


class _CoarsestLevel:
    """The coarsest level alone (a hierarchy partitioned down to it): its operator, buffers and dense pseudo-inverse, as
    mg.Multigrid holds its last level (the same struct fields, the same inverse)."""

    def __init__(self, A: DeviceCSR, ratio: float):
        from .mg import dense_inverse_csr
        dev = A.val.device
        d = A.diagonal()
        lmax = A.gershgorin(d)
        self.bounds = [(lmax / ratio, lmax)]
        self.A, self.diag = A, d
        self.coarse_inv, inv = dense_inverse_csr(A)
        self.coarse_dense = torch.from_numpy(np.ascontiguousarray(inv.T)).to(dev)
        self.work = [[torch.zeros(A.shape[0], dtype=torch.float64, device=dev) for _ in range(5)]]
        self._levels = (_lib.MgLevel * 1)()
        L = self._levels[0]
        L.nrows = A.shape[0]
        L.lmin, L.lmax = self.bounds[0]
        L.A, L.A_blocks, L.diag = A.cstruct(), A.blocks.cstruct(), d.data_ptr()
        L.R = L.P = _lib.Csr(0, 0, 0, None, None, None)
        L.R_blocks = L.P_blocks = _lib.RowBlocks(None, 0)
        L.x, L.t, L.r, L.d, L.b = (w.data_ptr() for w in self.work[0])


class _GlobalLevels:
    """LocalHierarchy's interface over a whole mg.Multigrid (every rank holds the global hierarchy)."""

    def __init__(self, g):
        self.g = g
        self.device, self.sizes, self.fields, self.n = g.device, g.sizes, g.fields, g.n
        self.nlevels, self.pre, self.post, self.cycles = g.nlevels, g.pre, g.post, g.cycles

    def _rows(self, M, rows):
        return M.extract(rows, torch.arange(M.shape[1], dtype=torch.int32, device=self.device), M.shape[1])

    def op_rows(self, l, rows):
        return self._rows(self.g.ops[l], rows)

    def R_rows(self, l, rows):
        return self._rows(self.g.R[l], rows)

    def P_rows(self, l, rows):
        return self._rows(self.g.P[l], rows)

    def diag_rows(self, l, rows):
        return self.g.diags[l][rows.long()].contiguous()

    def bounds(self, l, rows):
        return self.g.bounds[l]

    def replicated(self, P):
        return _Shifted(self.g, P)


class _Shifted:
    """Levels P .. end of a whole hierarchy, numbered from 0 (LocalHierarchy.replicated's form)."""

    def __init__(self, g, P):
        self.g, self.P = g, P
        self._levels = g._levels[P:]
        self.work = g.work[P:]
        self.bounds = g.bounds[P:]
        self.coarse_inv, self.coarse_dense = g.coarse_inv, g.coarse_dense


class PartitionedMultigrid:
    """A multigrid hierarchy (mg.Multigrid, built on every rank from the global operator -- setup only) split over a
    row partition for the partitioned Schur apply (solve.py:266 / 274's pointer, under north_star's row partition).

    Level l + 1's rows of rank k are [ceil(r0 / 2), ceil(r1 / 2)) of its level-l rows [r0, r1) (exact halving when
    the rows are even; a disjoint cover of the coarse grid in any case).  Levels [0, part_levels) are row-partitioned:
    their operator, restriction and prolongation rows extracted with the columns renumbered into the ghost layout
    (entry order kept), their vectors owned + ghost rows, ghost depths measured from the columns.  The restriction
    into level part_levels leaves each rank's rows of that level, all-gathered into the whole level; the coarser
    levels (and the dense coarsest inverse) run replicated on every rank.  Every operation is the one-GPU hierarchy's
    on the same operands: bit-identical to Multigrid.solve / the one-GPU apply.  Partitioning stops at the coarsest
    level, where a rank would hold fewer rows than the ghost depth, or below min_cells unknowns per rank."""

    def __init__(self, g, part: RowPartition, nfields: int, group=None, min_cells: int = 1 << 14,
                 max_part_levels: int | None = None):
        # g: a LocalHierarchy (this rank's rows only) or a whole mg.Multigrid (every rank holds it)
        g = g if isinstance(g, LocalHierarchy) else _GlobalLevels(g)
        self.g, self.part0, self.nf, self.group = g, part, nfields, group
        dev = g.device
        self.device = dev
        nl = g.nlevels
        self.parts = level_partitions(part, g.sizes)
        world = part.world

        def owned(l):
            return torch.from_numpy(self.parts[l].owned_rows(nfields).astype(np.int32)).to(dev)

        def depth(full, l):   # ghost rows of level l read by the rows `full` (global columns at level l)
            if world == 1:
                return 1
            q = self.parts[l]
            return ghost_depth(full.col_idx, q.n, q.r0, q.L)

        def reduce_max(v):
            if world == 1:
                return v
            import torch.distributed as dist
            t = torch.tensor([v], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            return int(t.item())

        self.h0 = reduce_max(max(1, depth(g.R_rows(0, owned(1)), 0)))   # level 0 ghosts the restriction reads
        self.h = [self.h0]
        P = nl - 1
        cap = nl - 1 if max_part_levels is None else max(1, min(nl - 1, max_part_levels))
        for l in range(1, nl - 1):
            q = self.parts[l]
            cells = nfields * q.n * q.n // world
            hl = reduce_max(max(1, depth(g.op_rows(l, owned(l)), l), depth(g.R_rows(l, owned(l + 1)), l),
                                depth(g.P_rows(l - 1, owned(l - 1)), l)))
            if l >= cap or cells < min_cells or q.min_rows < hl:
                P = l
                break
            self.h.append(hl)
        self.part_levels = P
        self._owned = owned

    def build(self, halos: _Halos, level0, diag0, h0: int, kind0: int | None = None, A0=None, cycles=None):
        """Local operators, vectors and the mpbp_mg struct.  level0: (x, t) iterate buffers of level 0 (owned + ghost
        rows at depth h0 >= self.h0; inside the Schur apply its own); diag0: level 0's owned diagonal; kind0: level 0's
        halo kind (the Schur apply's velocity / pressure kind; None: a new one); A0: level 0's local operator for the
        standalone solve (mpbp_mg_solve; None inside the Schur apply, whose level 0 is its own operator)."""
        g, nf, P, dev = self.g, self.nf, self.part_levels, self.device
        rep = g.replicated(P)   # levels P .. end, whole on every rank
        if h0 < self.h0:
            raise ValueError(f"level 0 ghost depth {h0} < the restriction's {self.h0}")
        self.h[0] = h0
        from .mg import sell_copy
        f64 = dict(dtype=torch.float64, device=dev)
        self.kinds, self.local, self.work = [], [], []
        for l in range(P):
            q = self.parts[l]
            self.kinds.append(halos.add_kind(q, nf, self.h[l]) if (l > 0 or kind0 is None) else kind0)
        gather_bounds = self.parts[P].bounds
        self.gather_kind = halos.add_gather(nf, self.parts[P].n, gather_bounds, self.part0.rank)
        self._levels = (_lib.MgLevel * g.nlevels)()
        empty_sell = _lib.Sell(0, 0, 0, 0, None, None, None, None)
        keep = []
        for l in range(g.nlevels):
            L = self._levels[l]
            L.pre, L.post = g.pre, g.post
            if l >= P:   # replicated: the whole level
                G = rep._levels[l - P]
                for name, _ in _lib.MgLevel._fields_:
                    setattr(L, name, getattr(G, name))
                L.lmin, L.lmax = rep.bounds[l - P]
                continue
            q = self.parts[l]
            rows = self._owned(l)
            L.lmin, L.lmax = g.bounds(l, rows)
            ext = q.n_ext(nf, self.h[l])
            cm = torch.from_numpy(q.colmap(nf, self.h[l])).to(dev)
            if l + 1 < P:
                qn = self.parts[l + 1]
                cm_next = torch.from_numpy(qn.colmap(nf, self.h[l + 1])).to(dev)
                ext_next = qn.n_ext(nf, self.h[l + 1])
            else:
                ncoarse = nf * g.sizes[l + 1] ** 2
                cm_next, ext_next = torch.arange(ncoarse, dtype=torch.int32, device=dev), ncoarse

            def local(M, cmap, ncols):   # all rows of M (global columns) with the columns into the ghost layout
                return M.extract(torch.arange(M.shape[0], dtype=torch.int32, device=dev), cmap, ncols)
            R = local(g.R_rows(l, self._owned(l + 1)), cm, ext)
            Pm = local(g.P_rows(l, rows), cm_next, ext_next)
            own = q.n_owned(nf)
            L.nrows = own
            if l == 0:
                L.A = A0.cstruct() if A0 is not None else _lib.Csr(0, 0, 0, None, None, None)
                L.A_blocks = A0.blocks.cstruct() if A0 is not None else _lib.RowBlocks(None, 0)
                L.diag = diag0.data_ptr()
                SA = sell_copy(A0) if A0 is not None else None
                L.A_sell = SA.cstruct() if SA is not None else empty_sell
                keep += [A0, SA, diag0]
                x, t = level0
                r = torch.zeros(ext, **f64)
                d, bb = torch.zeros(own, **f64), torch.zeros(own, **f64)
            else:
                A = local(g.op_rows(l, rows), cm, ext)
                dg = g.diag_rows(l, rows)
                L.A, L.A_blocks, L.diag = A.cstruct(), A.blocks.cstruct(), dg.data_ptr()
                SA = sell_copy(A)
                L.A_sell = SA.cstruct() if SA is not None else empty_sell
                keep += [A, dg, SA]
                x, t, r = (torch.zeros(ext, **f64) for _ in range(3))
                d, bb = torch.zeros(own, **f64), torch.zeros(own, **f64)
            SR, SP = sell_copy(R), sell_copy(Pm)
            L.R, L.R_blocks, L.P, L.P_blocks = R.cstruct(), R.blocks.cstruct(), Pm.cstruct(), Pm.blocks.cstruct()
            L.R_sell = SR.cstruct() if SR is not None else empty_sell
            L.P_sell = SP.cstruct() if SP is not None else empty_sell
            keep += [R, Pm, SR, SP]
            L.x, L.t, L.r, L.d, L.b = (v.data_ptr() for v in (x, t, r, d, bb))
            L.halo_kind = self.kinds[l]
            L.part_r0, L.part_h = q.r0, self.h[l]   # (the matrix-free level 1's owned window, k_gal1 / k_gal1p)
            self.work.append((x, t, r, d, bb))
            halos.register(x, t, r, d, bb)
        # the gather level's r (the rank's rows, written by the restriction) and b (the whole level) are the global
        # level's full-size buffers
        Gw = rep.work[0]
        halos.register(*Gw)
        self._keep = keep + [rep]
        self._halos = halos
        self._mg = _lib.Mg(g.nlevels, g.cycles if cycles is None else cycles,
                           ctypes.cast(self._levels, ctypes.POINTER(_lib.MgLevel)),
                           rep.coarse_inv.cstruct(), rep.coarse_inv.blocks.cstruct(),
                           rep.coarse_dense.data_ptr() if rep.coarse_dense is not None else None,
                           P, self.gather_kind, halos.fn, halos.ctx, halos.gather_fn)
        from .mg import set_transfer_kinds
        set_transfer_kinds(self._mg, g.fields, g.n)   # (matrix-free transfers on the replicated levels only)
        return self

    def cstruct(self):
        return self._mg


def _dist_info(group):
    import torch.distributed as dist
    return dist, dist.get_world_size(group), dist.get_rank(group), dist.get_backend(group)


def _phase_clock(out: dict):
    """stamp(name): with MPBP_SETUP_TIMING=1, synchronise the device and record the seconds since the previous stamp
    under `name` in `out`; otherwise nothing (no extra synchronisation in production setups)."""
    if os.environ.get("MPBP_SETUP_TIMING", "0") != "1":
        return lambda name: None
    import time
    torch.cuda.synchronize()
    last = [time.perf_counter()]

    def stamp(name):
        torch.cuda.synchronize()
        t = time.perf_counter()
        out[name] = out.get(name, 0.0) + (t - last[0])
        last[0] = t
    return stamp


class DistributedMatrix:
    """A row-partitioned operator of the MAC-grid system: the operator matvec b = A u of apply.py:72 and the FGMRES
    operator of solve.py:285 (A @ xk, solve.py:166) over the ranks of `group`, one per GPU.

    Rank k holds the rows of grid rows [r0, r1) of every one of `nfields` stacked n x n fields (A: the 5 fields
    [u_n, v_n, u_s, v_s, p]), columns renumbered into the owned + ghost ("ext") layout (DeviceCSR.extract keeps each
    row's entry order: every local row sum is the global one, bit for bit).  apply(x) takes and returns the rank's
    owned entries: x is copied into the ext buffer, the ghost rows are exchanged (RCCL neighbour point-to-point over
    xGMI -- overlap=True: on the halo's own high-priority stream, forked before and joined after the interior rows'
    SpMV, so the transfer overlaps it), the interior rows (no ghost column) run on the CSR kernel meanwhile and the
    boundary rows after the join.  With the gloo backend the ghosts are host-staged (HaloExchanger)."""

    def __init__(self, M: DeviceCSR, n: int, nfields: int, group=None, halo: str = "auto", overlap: bool = True,
                 self_halo: bool = False, owned_rows: bool = False):
        """M: the global operator, or (owned_rows=True) just this rank's rows of it, in owned order, with global
        columns (MultiphaseBlockPreconditioner.assemble_rows: rank-local setup)."""
        dist, world, rank, backend = _dist_info(group)
        dev = M.device
        N_all = nfields * n * n
        self.part = part = RowPartition(n, world, rank, ghosts=bool(self_halo))
        if M.shape != ((part.n_owned(nfields) if owned_rows else N_all), N_all):
            raise ValueError(f"operator {M.shape} is not {'this rank' + chr(39) + 's rows of ' if owned_rows else ''}"
                             f"{nfields} fields of a {n} x {n} grid")
        self.nfields = nfields
        self.partitioned = part.ghosts
        self.halo_impl = halo if halo != "auto" else ("rccl" if backend == "nccl" else "torch")
        rows = torch.from_numpy(part.owned_rows(nfields).astype(np.int32)).to(dev)
        if owned_rows:
            full, rows = M, torch.arange(M.shape[0], dtype=torch.int32, device=dev)
        else:
            full = M.extract(rows, torch.arange(M.shape[1], dtype=torch.int32, device=dev), M.shape[1])
        self.h = max(1, ghost_depth(full.col_idx, n, part.r0, part.L) if world > 1 else 1)
        del full
        self.n_own = part.n_owned(nfields)
        self.n_ext = part.n_ext(nfields, self.h)
        self.shape = (self.n_own, self.n_own)
        if owned_rows and not self.partitioned:
            raise ValueError("owned_rows=True needs a row partition")
        self.A = M.extract(rows, torch.from_numpy(part.colmap(nfields, self.h)).to(dev), self.n_ext) \
            if self.partitioned else M
        if self.partitioned and world > 1:
            inner, bnd = boundary_ranges(self.A.row_ptr, self.A.col_idx, self.n_own)
        elif self.partitioned:   # one rank exchanging with itself: every row with a wrapped neighbour reads ghosts
            inner, bnd = boundary_ranges(self.A.row_ptr, self.A.col_idx, self.n_own)
        else:
            inner, bnd = [(0, self.n_own)], []
        self.blk_in = self.A.plan_blocks(rows=inner) if inner else None
        self.blk_bd = self.A.plan_blocks(rows=bnd) if bnd else None
        self.xe = torch.zeros(self.n_ext, dtype=torch.float64, device=dev)
        self._rccl = self._ex = None
        if self.partitioned:
            if self.halo_impl == "rccl":
                # its own communicator: its exchanges run eagerly on the halo object's side stream (overlap), the
                # preconditioner's in order on the caller's stream inside a replayed graph -- the two are never mixed
                # on one communicator
                self._rccl = RcclHalo(part, 1, 1, group, overlap=False, share=False)
                self.kind = self._rccl.add_kind(part, nfields, self.h, overlap=overlap)
            else:
                self._ex = HaloExchanger(part, nfields, self.h, dev, group)

    @property
    def device(self):
        return self.xe.device

    def apply(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        assert x.is_cuda and x.dtype == torch.float64 and x.numel() == self.n_own
        if out is None:
            out = torch.empty(self.n_own, dtype=torch.float64, device=x.device)
        if not self.partitioned:
            return self.A.matvec(x, out=out)
        self.xe[: self.n_own].copy_(x)
        st = stream_handle()
        if self._rccl is not None:
            lib().mpbp_halo_exchange(self._rccl.handle, self.kind, ptr(self.xe), _lib.HALO_BEGIN, st)
        else:
            self._ex.begin(self.xe)
        if self.blk_in is not None:
            self.A.matvec(self.xe, out=out, blocks=self.blk_in)
        if self._rccl is not None:
            lib().mpbp_halo_exchange(self._rccl.handle, self.kind, ptr(self.xe), _lib.HALO_END, st)
        else:
            self._ex.end(self.xe)
        if self.blk_bd is not None:
            self.A.matvec(self.xe, out=out, blocks=self.blk_bd)
        if self._rccl is not None:
            self._rccl.check()
        return out

    matvec = apply

    def close(self):
        if self._rccl is not None:
            self._rccl.close()
            self._rccl = None

    def local_to_global_rows(self):
        return self.part.owned_rows(self.nfields)


def _csr_vstack(A: DeviceCSR, B: DeviceCSR) -> DeviceCSR:
    """The rows of A, then the rows of B (same column count), as one CSR."""
    rp = torch.cat([A.row_ptr[:-1], B.row_ptr + A.nnz])
    return DeviceCSR(rp.contiguous(), torch.cat([A.col_idx, B.col_idx]), torch.cat([A.val, B.val]),
                     (A.shape[0] + B.shape[0], A.shape[1]))


def _q13_block(Q: DeviceCSR, n: int, part, group, red_dev):
    """(n, vals, symmetric) for a row partition: Gt_F_G's diamond over grid rows r0 - 2 .. r0 + L - 1 (Q: those rows
    with global columns, mpbp_q13_build_rows) and whether the product is symmetric to 1e-14 of its largest entry over
    every rank's owned rows (slot s at a cell against slot 12 - s at its neighbour (dr_s, dc_s) -- mpbp_q13_asymmetry's
    test, reduced over the ranks).  None when Q's rows are not the 13-point diamond."""
    import torch.distributed as dist
    L = part.L
    vals = torch.empty(13 * (L + 2) * n, dtype=torch.float64, device=Q.device)
    if lib().mpbp_q13_build_rows(ctypes.byref(Q.cstruct()), n, part.r0 - 2, ptr(vals), stream_handle()) != 0:
        ok = torch.tensor([0.0], dtype=torch.float64, device=red_dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MAX, group=group)   # (the same collective on every rank)
        dist.all_reduce(ok, op=dist.ReduceOp.MAX, group=group)
        return None
    V = vals.view(13, L + 2, n)
    amax = V[:, 2:, :].abs().max()
    asym = torch.zeros((), dtype=torch.float64, device=Q.device)
    dr = (-2, -1, -1, -1, 0, 0)
    dc = (0, -1, 0, 1, -2, -1)
    for s in range(6):
        nb = torch.roll(V[12 - s, 2 + dr[s]: 2 + dr[s] + L, :], shifts=-dc[s], dims=1)
        asym = torch.maximum(asym, (V[s, 2:, :] - nb).abs().max())
    a = torch.stack([asym, amax]).to(red_dev)
    dist.all_reduce(a[0:1], op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(a[1:2], op=dist.ReduceOp.MAX, group=group)
    a = a.cpu()
    return n, vals, bool(a[0] <= 1e-14 * a[1])


class DistributedSchurPreconditioner(PlanProfiling):
    """The approximate-commutator apply over a row partition of the grid (one rank per GPU).

    Every rank assembles the global operators in its own HBM (setup only), keeps its rows with
    columns renumbered into the owned+ghost layout, and runs ``mpbp_schur_apply`` with halo
    callbacks; v and the result hold the rank's owned unknowns [u_n, v_n, u_s, v_s, p] rows r0..r1.
    Inner solves: Jacobi / Chebyshev (the communication-avoiding schedule by default) or multigrid ("mg": one
    PartitionedMultigrid per inner inverse, ghost rows exchanged per operator, the coarse levels replicated).

    Graph capture (``capture``) needs the in-order RCCL halo.  A communicator whose exchanges were captured is kept
    until the process exits (``close`` does not destroy it: with RCCL 2.26.6 ncclCommDestroy never returns once a
    graph holding its point-to-point kernels has been instantiated and destroyed; csrc/halo.cpp).
    """

    def __init__(self, n, xi, eta_n, eta_s, c=1.0, d_u=-1.0, inner_F=None, inner_P=None, group=None,
                 device=None, layout="sell", f_mode="auto", pg_mode="auto", halo="auto", self_halo=False,
                 halo_overlap=False, ca="auto", fuse_g=True, mg_min_cells=1 << 14, mg_part_levels=None,
                 local_products=True, numerics="exact", kernel_opts=None):
        import torch.distributed as dist
        from .preconditioner import MultiphaseBlockPreconditioner
        from .solve import InnerSolver, _check_numerics
        self.numerics = _check_numerics(numerics)
        # this preconditioner's kernel choices (process defaults now + overrides): tolerance mode reads Gt_F_G's
        # symmetric half over the rank's row block (q13_sym, as one GPU); q13_mf is one-GPU only
        self.kernel_opts = _lib.kernel_opts(kernel_opts)
        # setup phase timings (MPBP_SETUP_TIMING=1: synchronise and stamp each phase; tools/setup_timing.py)
        self.setup_phases = {}
        _stamp = _phase_clock(self.setup_phases)
        dev = torch.device(device or "cuda")
        self.device = dev
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        # self_halo: a single rank still runs the partitioned apply, its ghost rows filled by the periodic
        # self-exchange (exercises the interior / boundary launches and the halo path on one GPU)
        self.part = part = RowPartition(n, world, rank, ghosts=bool(self_halo))
        self.partitioned = part.ghosts
        if halo not in ("auto", "rccl", "torch"):
            raise ValueError("halo must be 'auto', 'rccl' or 'torch'")
        backend = dist.get_backend(group)
        self.halo_impl = halo if halo != "auto" else ("rccl" if backend == "nccl" else "torch")
        bp = MultiphaseBlockPreconditioner(n, xi, eta_n, eta_s, device=dev)
        rows_u = torch.from_numpy(part.owned_rows(N_VEL_FIELDS).astype(np.int32)).to(dev)
        rows_p = torch.from_numpy(part.owned_rows(N_P_FIELDS).astype(np.int32)).to(dev)
        ik_f, ik_p = inner_F or InnerSolver(), inner_P or InnerSolver()
        # the commutator products: only this rank's pressure rows of Gt_G and Gt_F_G (a product's row depends on that
        # row of D alone: the same bits as the global product's row, for a 1 / world share of the SpGEMM work);
        # multigrid inner solves form their levels from this rank's band of rows too (LocalHierarchy)
        self.local_products = bool(local_products) and world > 1
        akw = dict(c=c, d_u=d_u)
        Gs = None
        if self.local_products:
            # rank-local setup (preconditioner.py:299-341 row by row): F, D, G assembled on this rank's rows only
            # (mpbp_stokes_*_rows, the global assembly's rows bit for bit), the products' right operands on the velocity
            # rows a product row can reach -- grid rows within `sup` of the owned ones (the CA schedule's ghost depths
            # included) -- in global row numbering; setup memory and work O(N / world + ghosts) instead of O(N)
            st_F, st_D, st_G = bp.stencils(**akw)
            F = bp.assemble_rows(_lib.OP_F, rows_u, **akw)
            D = bp.assemble_rows(_lib.OP_D, rows_p, **akw)
            G = bp.assemble_rows(_lib.OP_G, rows_u, **akw)
            F.stencil, D.stencil, G.stencil = st_F, st_D, st_G
            _stamp("assemble_owned_rows")
            sweeps = lambda k: k.sweeps if k.kind in ("jacobi", "chebyshev") else 1   # noqa: E731
            sup = min(n, sweeps(ik_f) + sweeps(ik_p) + 2)
            grid_rows = np.unique(np.arange(part.r0 - sup, part.r1 + sup) % n) if part.L + 2 * sup < n \
                else np.arange(n)
            sup_u = np.sort(np.concatenate([f * part.N + (r * n + np.arange(n)) for f in range(N_VEL_FIELDS)
                                            for r in grid_rows]))
            sup_u = torch.from_numpy(sup_u.astype(np.int32)).to(dev)
            Fs = bp.assemble_rows(_lib.OP_F, sup_u, global_shape=True, **akw)
            Gs = bp.assemble_rows(_lib.OP_G, sup_u, global_shape=True, **akw)
            _stamp("assemble_support_rows")
            GtG, GtFG = bp.commutator_products(Fs, D, Gs)   # this rank's pressure rows, global columns
            _stamp("commutator_products")
            GtG.stencil = _gtg_stencil(D, G)
            # tolerance mode: the two pressure grid rows above the owned block too (their products' rows, bit for bit
            # the global product's), so the symmetric-half read has the lower slots of the first owned rows
            q_rows = None
            if self.numerics == "fast" and part.ghosts and part.L < n:
                q_rows = GtFG
                for k in (1, 2):   # (one grid row per assembly: the wrapped rows need not ascend)
                    row = torch.from_numpy((((part.r0 - k) % n) * n + np.arange(n)).astype(np.int32)).to(dev)
                    D1 = bp.assemble_rows(_lib.OP_D, row, **akw)
                    q_rows = _csr_vstack(spgemm(spgemm(D1, Fs, alpha=-1.0), Gs, alpha=1.0), q_rows)
                del D1
            del Fs
        else:
            _, _, F, D, G = bp.get_big_A_matrix(**akw)
            _stamp("assemble_global")
            GtG, GtFG = bp.commutator_products(F, D, G)
            _stamp("commutator_products")
            q_rows = None
            if self.numerics == "fast" and part.ghosts:   # grid rows r0 - 2 .. r0 + L - 1 of the global product
                blk = np.concatenate([((part.r0 + k) % n) * n + np.arange(n) for k in range(-2, part.L)]).astype(np.int32)
                q_rows = GtFG.extract(torch.from_numpy(blk).to(dev),
                                      torch.arange(GtFG.shape[1], dtype=torch.int32, device=dev), GtFG.shape[1])
        # Gt_F_G's diamond over the rank's row block, read from its symmetric upper half (k_q13p) when the product is
        # symmetric to 1e-14 of its largest entry -- decided over all ranks, as one GPU decides over the whole grid
        self.q13 = None
        if q_rows is not None and n >= 5:
            self.q13 = _q13_block(q_rows, n, part, group, dev if backend == "nccl" else "cpu")
            if self.q13 is None or not self.q13[2]:
                self.kernel_opts.q13_sym = 0
        else:
            self.kernel_opts.q13_sym = 0
        del q_rows
        lp = self.local_products
        if f_mode not in ("auto", "stencil", "assembled"):
            raise ValueError("f_mode must be 'auto', 'stencil' or 'assembled'")
        if f_mode == "stencil" and F.stencil is None:
            raise ValueError("f_mode='stencil' needs n >= 3")
        self.f_stencil = F.stencil if f_mode in ("auto", "stencil") else None
        self.pg_stencil = _pg_stencil(D, G, GtG, self.f_stencil, pg_mode)
        # inner-solver bounds from the global operators: identical on every rank (rank-local: the Gershgorin bound is the
        # maximum of the ranks' row bounds -- the same maximum, exactly)
        def global_bound(M, rows):
            t = torch.tensor([M.gershgorin(_row_diagonal(M, rows))], dtype=torch.float64,
                             device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            return float(t.item())
        if lp and ik_f.kind == "chebyshev" and ik_f.lmax is None:
            ik_f = InnerSolver("chebyshev", ik_f.sweeps, ik_f.lmin, global_bound(F, rows_u), ik_f.ratio)
        self.inner_F = ik_f.resolve(F, None if lp else F.diagonal())
        if self.local_products:
            ip = ik_p
            if ip.kind == "chebyshev" and ip.lmax is None:
                ip = InnerSolver("chebyshev", ip.sweeps, ip.lmin, global_bound(GtG, rows_p), ip.ratio)
            self.inner_P = ip.resolve(GtG, None)
        else:
            self.inner_P = (inner_P or InnerSolver()).resolve(GtG, GtG.diagonal())
        mg_any = "mg" in (self.inner_F.kind, self.inner_P.kind)
        _stamp("inner_bounds")

        def reach(M, rows, local=False):
            sub = M if local else M.extract(rows, torch.arange(M.shape[1], dtype=torch.int32, device=dev), M.shape[1])
            return halo_reach(sub.row_ptr, sub.col_idx, rows, n)

        q = reach(GtFG, rows_p, lp)
        self.h_u = max(1, reach(F, rows_u, lp), reach(D, rows_p, lp))
        self.h_p = max(1, reach(G, rows_u, lp), reach(GtG, rows_p, lp), q)
        # multigrid inner solves: the global hierarchies (every rank, setup only), split over the partition; level 0's
        # ghost layout must also serve the restriction's reach
        self.mg_F = self.mg_P = None
        if mg_any:
            from .mg import FIELDS_PRESSURE, FIELDS_VELOCITY
            if ca is True:
                raise ValueError("ca=True needs Jacobi / Chebyshev inner solves (multigrid exchanges per operator)")
            kw = dict(group=group, min_cells=mg_min_cells, max_part_levels=mg_part_levels)

            def local_mg(ik, fields):
                # this rank's band of level 0 (mg_bands), then its Galerkin levels (LocalHierarchy): no global operator
                from .mg import level_sizes
                sizes = level_sizes(n, ik.coarsest)
                cap = mg_part_cap(sizes, part, len(fields), mg_min_cells, mg_part_levels)
                S = mg_bands(sizes, fields, part, cap, dev)
                _stamp("mg_bands")
                if fields is FIELDS_VELOCITY:
                    A0 = bp.assemble_rows(_lib.OP_F, S[0], **akw)
                else:   # Gt_G's band rows = (-D) G on them, G on the velocity rows those rows of D reach
                    Db = bp.assemble_rows(_lib.OP_D, S[0], **akw)
                    Gb = bp.assemble_rows(_lib.OP_G, torch.unique(Db.col_idx), global_shape=True, **akw)
                    A0 = spgemm(Db, Gb, alpha=-1.0)
                    del Db, Gb
                _stamp("mg_band_level0")
                return LocalHierarchy(A0, S, sizes, fields, part, group, pre=ik.pre, post=ik.post,
                                      cycles=int(ik.sweeps), ratio=ik.smooth_ratio, coarsest=ik.coarsest, stamp=_stamp)
            if self.inner_F.kind == "mg":
                gF = local_mg(self.inner_F, FIELDS_VELOCITY) if lp else \
                    self.inner_F.multigrid(F, n, FIELDS_VELOCITY, F.diagonal())
                self.mg_F = PartitionedMultigrid(gF, part, N_VEL_FIELDS, **kw) if self.partitioned else gF
            if self.inner_P.kind == "mg":
                gP = local_mg(self.inner_P, FIELDS_PRESSURE) if lp else \
                    self.inner_P.multigrid(GtG, n, FIELDS_PRESSURE, GtG.diagonal())
                self.mg_P = PartitionedMultigrid(gP, part, N_P_FIELDS, **kw) if self.partitioned else gP
            if isinstance(self.mg_F, PartitionedMultigrid):
                self.h_u = max(self.h_u, self.mg_F.h0)
            if isinstance(self.mg_P, PartitionedMultigrid):
                self.h_p = max(self.h_p, self.mg_P.h0)
        _stamp("halo_reach_and_multigrid")
        # communication-avoiding schedule (mpbp_schur_plan.ca): v's halo and x_b's halo only, deep enough for
        # every matrix-free operator to also compute the ghost rows its successors read
        if ca not in ("auto", True, False):
            raise ValueError("ca must be 'auto', True or False")
        self.ca, self.ca_q = False, q
        if ca and not mg_any and part.ghosts and self.f_stencil is not None and self.pg_stencil is not None:
            sf, sp = self.inner_F.sweeps - 1, self.inner_P.sweeps - 1
            hu, hp = q + sp + 1 + sf, max(q + sp, sf + 1 + sp, q)
            if max(hu, hp) <= part.min_rows:
                self.ca = True
                self.h_u, self.h_p = max(self.h_u, hu), max(self.h_p, hp)
            elif ca is True:
                raise ValueError(f"ca=True needs {max(hu, hp)} grid rows per rank, the smallest has {part.min_rows}")
        elif ca is True:
            raise ValueError("ca=True needs a row partition and the matrix-free F, D, G, Gt_G")
        # CA schedule: the second F solve recomputes G x_p inside its sweeps from x_p's ghost rows (no G launch)
        self.fuse_g = bool(fuse_g and self.ca and self.inner_F.kind == "chebyshev" and self.inner_F.sweeps >= 2)
        nu, np_ = part.n_owned(N_VEL_FIELDS), part.n_owned(N_P_FIELDS)
        nu_ext, np_ext = part.n_ext(N_VEL_FIELDS, self.h_u), part.n_ext(N_P_FIELDS, self.h_p)
        cm_u = torch.from_numpy(part.colmap(N_VEL_FIELDS, self.h_u)).to(dev)
        cm_p = torch.from_numpy(part.colmap(N_P_FIELDS, self.h_p)).to(dev)
        if self.ca:
            gp_rows = torch.from_numpy(part.ext_rows(N_P_FIELDS, self.h_p).astype(np.int32)).to(dev)
            if lp:   # F's diagonal on the owned + ghost velocity rows, from those rows alone
                gu = torch.from_numpy(part.ext_rows(N_VEL_FIELDS, self.h_u).astype(np.int32)).to(dev)
                self.diag_F_ext = _row_diagonal(bp.assemble_rows(_lib.OP_F, gu, **akw), gu)
            else:
                diag_F_glob = F.diagonal()
            if lp:   # Gt_G's diagonal on the owned + ghost pressure rows, from those rows of the product alone
                D_ext = bp.assemble_rows(_lib.OP_D, gp_rows, **akw)
                self.diag_P_ext = _row_diagonal(spgemm(D_ext, Gs, alpha=-1.0), gp_rows)
                del D_ext
            else:
                diag_P_glob = GtG.diagonal()
        _stamp("ca_ghost_diagonals")
        if lp:   # already this rank's rows, in owned order
            own_u = torch.arange(rows_u.numel(), dtype=torch.int32, device=dev)
            own_p = torch.arange(rows_p.numel(), dtype=torch.int32, device=dev)
            self.F = F.extract(own_u, cm_u, nu_ext)
            self.D = D.extract(own_p, cm_u, nu_ext)
            self.G = G.extract(own_u, cm_p, np_ext)
            self.GtG = GtG.extract(own_p, cm_p, np_ext)
            self.GtFG = GtFG.extract(own_p, cm_p, np_ext)
        else:
            self.F = F.extract(rows_u, cm_u, nu_ext)
            self.D = D.extract(rows_p, cm_u, nu_ext)
            self.G = G.extract(rows_u, cm_p, np_ext)
            self.GtG = GtG.extract(rows_p, cm_p, np_ext)
            self.GtFG = GtFG.extract(rows_p, cm_p, np_ext)
        del F, D, G, GtG, GtFG, Gs, bp
        torch.cuda.empty_cache()
        self.nu, self.np, self.nu_ext, self.np_ext = nu, np_, nu_ext, np_ext
        self.shape = (nu + np_, nu + np_)
        self.diag_F = self.F.diagonal()
        self.diag_P = self.GtG.diagonal()
        if self.ca and not lp:   # diagonals on owned + ghost rows (the CA schedule's ghost-row sweeps stage x0)
            gu = torch.from_numpy(part.ext_rows(N_VEL_FIELDS, self.h_u)).to(dev)
            self.diag_F_ext = diag_F_glob[gu].contiguous()
            gp = torch.from_numpy(part.ext_rows(N_P_FIELDS, self.h_p)).to(dev)
            self.diag_P_ext = diag_P_glob[gp].contiguous()
            del diag_P_glob, diag_F_glob

        _stamp("extract_ghost_layout")
        mats = {"F": (self.F, nu), "D": (self.D, nu), "G": (self.G, np_), "P": (self.GtG, np_),
                "Q": (self.GtFG, np_)}
        self._pieces = {}
        self.layout = layout
        for key, (M, n_own_cols) in mats.items():
            inner, bnd = boundary_ranges(M.row_ptr, M.col_idx, n_own_cols) if world > 1 else \
                ([(0, M.shape[0])], [])
            if layout == "sell":
                S = M.to_sell(inner + bnd)
                n_in = sum((b - a + 63) // 64 for a, b in inner)
                self._pieces[key] = (S, S.sub(0, n_in), S.sub(n_in, S.nslices - n_in))
            else:
                self._pieces[key] = (M.plan_blocks(rows=inner) if inner else None,
                                     M.plan_blocks(rows=bnd) if bnd else None)
        _stamp("sell_layouts")
        f64 = dict(dtype=torch.float64, device=dev)
        self._wu = [torch.zeros(nu_ext, **f64) for _ in range(4)]
        self._wu_owned = torch.zeros(nu, **f64)
        self._wp = [torch.zeros(np_ext, **f64) for _ in range(7)]
        self._wu_ext = torch.zeros(nu_ext if self.ca else 0, **f64)
        self._rccl = None
        self._halos = None
        if self.partitioned:
            if self.halo_impl == "rccl":
                self._rccl = RcclHalo(part, self.h_u, self.h_p, group, overlap=halo_overlap)
            self._halos = _Halos(self.halo_impl, self._rccl, group, dev)
            if self._rccl is None:
                self._halos.add_kind(part, N_VEL_FIELDS, self.h_u, kind=_lib.VEC_VELOCITY)
                self._halos.add_kind(part, N_P_FIELDS, self.h_p, kind=_lib.VEC_PRESSURE)
            self._halos.register(*self._wu, *self._wp, *([self._wu_ext] if self.ca else []))
            self._cb = self._halos.fn
            # multigrid under the partition: level 0 is the apply's own F / Gt_G with its ping / pong buffers
            if isinstance(self.mg_F, PartitionedMultigrid):
                self.mg_F.build(self._halos, (self._wu[1], self._wu[2]), self.diag_F, self.h_u, kind0=_lib.VEC_VELOCITY)
                _stamp("mg_build_F")
            if isinstance(self.mg_P, PartitionedMultigrid):
                self.mg_P.build(self._halos, (self._wp[4], self._wp[5]), self.diag_P, self.h_p, kind0=_lib.VEC_PRESSURE)
                _stamp("mg_build_P")
        else:
            self._cb = _lib.HALO_FN()
        _stamp("halo_and_workspace")
        self._prof = None
        self._plan = self._make_plan(world)
        _stamp("plan")

    def _make_plan(self, world):
        p = _lib.SchurPlan()
        p.nu, p.np, p.nu_ext, p.np_ext = self.nu, self.np, self.nu_ext, self.np_ext
        p.F, p.D, p.G = self.F.cstruct(), self.D.cstruct(), self.G.cstruct()
        p.GtG, p.GtFG = self.GtG.cstruct(), self.GtFG.cstruct()
        empty_b = _lib.RowBlocks(None, 0)
        empty_s = _lib.Sell(0, 0, 0, 0, None, None, None, None)
        p.use_sell = 1 if self.layout == "sell" else 0
        for key in "FDGPQ":
            piece = self._pieces[key]
            if self.layout == "sell":
                setattr(p, key + "s_int", piece[1].cstruct())
                setattr(p, key + "s_bnd", piece[2].cstruct())
                setattr(p, key + "_int", empty_b)
                setattr(p, key + "_bnd", empty_b)
            else:
                setattr(p, key + "_int", piece[0].cstruct() if piece[0] else empty_b)
                setattr(p, key + "_bnd", piece[1].cstruct() if piece[1] else empty_b)
                setattr(p, key + "s_int", empty_s)
                setattr(p, key + "s_bnd", empty_s)
        p.diag_F, p.diag_P = self.diag_F.data_ptr(), self.diag_P.data_ptr()
        p.inner_F, p.inner_P = self.inner_F.cstruct(), self.inner_P.cstruct()
        for i, t in enumerate(self._wu):
            p.wu[i] = t.data_ptr()
        p.wu_owned = self._wu_owned.data_ptr()
        for i, t in enumerate(self._wp):
            p.wp[i] = t.data_ptr()
        p.f_stencil = 1 if self.f_stencil is not None else 0
        p.pg_stencil = 1 if self.pg_stencil is not None else 0
        if self.f_stencil is not None:
            st = self.f_stencil
            p.f_prm = st.prm
            p.f_cell, p.f_uface, p.f_vface = st.cell.data_ptr(), st.uface.data_ptr(), st.vface.data_ptr()
        elif self.pg_stencil is not None:
            p.f_prm, p.f_cell = self.pg_stencil.prm, self.pg_stencil.cell.data_ptr()
        # velocity (F, D) and pressure (G, Gt_G) input partitions of the stencil operators
        ghost = self.partitioned
        p.f_part = _lib.RowPart(self.part.r0, self.part.L, self.h_u if ghost else 0, 0)
        p.p_part = _lib.RowPart(self.part.r0, self.part.L, self.h_p if ghost else 0, 0)
        p.halo = self._cb
        p.halo_ctx = self._rccl.handle if self._rccl is not None else None
        if self.mg_F is not None:
            p.mg_F = ctypes.pointer(self.mg_F.cstruct())
        if self.mg_P is not None:
            p.mg_P = ctypes.pointer(self.mg_P.cstruct())
        # the in-order RCCL schedule gains nothing from splitting rows around the exchange: exchange first,
        # then one launch per sweep
        p.halo_first = 1 if (self._rccl is not None and not self._rccl.overlap) else 0
        p.ca, p.ca_reach_q = (1 if self.ca else 0), self.ca_q
        if self.q13 is not None:
            p.q13, p.q13_n = self.q13[1].data_ptr(), self.q13[0]
        p.fuse_g = 1 if self.fuse_g else 0
        p.f_numerics = _lib.NUMERICS_FAST if self.numerics == "fast" else _lib.NUMERICS_EXACT
        p.opts = ctypes.pointer(self.kernel_opts)
        if self.ca:
            if self._rccl is not None and not self._rccl.overlap:   # v's two halves in one RCCL group
                p.halo_pair = self._rccl.pair_fn
            p.wu_ext = self._wu_ext.data_ptr()
            p.diag_F_ext, p.diag_P_ext = self.diag_F_ext.data_ptr(), self.diag_P_ext.data_ptr()
        p.prof_events = None
        p.prof_capacity = 0
        p.prof_count = ctypes.POINTER(ctypes.c_int32)()
        return p

    def sell_of(self, key):
        """The SELL-64 copy (interior + boundary slices) of F / D / G / P / Q, or None (CSR layout)."""
        return self._pieces[key][0] if self.layout == "sell" else None

    def apply(self, v: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        assert v.is_cuda and v.dtype == torch.float64 and v.numel() == self.nu + self.np
        if out is None:
            out = torch.empty_like(v)
        check(lib().mpbp_schur_apply(ctypes.byref(self._plan), ptr(v), ptr(out), stream_handle()))
        # every exchange and gather of the apply (its own halos and the partitioned multigrid levels') reports through
        # _Halos: the RCCL object's status, or the first exception a host-staged callback latched
        if self._halos is not None:
            self._halos.check()
        return out

    def capture(self, v: torch.Tensor, out: torch.Tensor):
        """Capture one apply(v, out) into a hipGraph.  Partitioned applies need the RCCL halo in order on the
        apply stream (the exchange is then a gather kernel plus one RCCL group of point-to-point calls, which
        RCCL records into the graph); the capture runs in thread-local error mode so that RCCL's proxy thread
        may keep calling HIP.  The torch halo (host-staged gloo collectives between kernels) cannot be
        captured."""
        if self.partitioned and (self._rccl is None or self._rccl.overlap):
            raise NotImplementedError("graph capture of a partitioned apply needs the in-order RCCL halo")
        return _capture(self, v, out, capture_error_mode="thread_local" if self.partitioned else "global")

    def close(self):
        if self._rccl is not None:
            self._rccl.close()
            self._rccl = None

    def local_to_global_rows(self):
        """Global ids (in the [u_n, v_n, u_s, v_s, p] numbering) of this rank's v / out entries."""
        return np.concatenate([self.part.owned_rows(N_VEL_FIELDS),
                               4 * self.part.N + self.part.owned_rows(N_P_FIELDS)])


def solve_distributed(n, xi, etan, etas, c=1.0, d=-1.0, b_vec=None, inner_F=None, inner_P=None, tol=1e-8,
                      maxiter=150, restrt=None, group=None, self_halo=False, keep_operators=False, **pc_kw):
    """solve.py:240-286 over a row partition (one rank per GPU): FGMRES (solve.fgmres over `group`) on the partitioned
    operator A (DistributedMatrix) with the partitioned approximate-commutator preconditioner
    (DistributedSchurPreconditioner).  b_vec: the global right-hand side on the host (default: the manufactured problem
    of solve.py:52-80).  The solve is the one-GPU solve's, bit for bit (reproducible inner products).  Returns a dict:
    x_local (this rank's rows of the iterate, CUDA), rows (their global ids), info, residuals, A, M.  Unless
    keep_operators, A and M are closed before the return (their RCCL communicators destroyed here, at the same point on
    every rank, also when the solve raises -- not whenever the garbage collector of each rank gets to them)."""
    import torch.distributed as dist
    from .preconditioner import MultiphaseBlockPreconditioner
    from .solve import fgmres
    from .utils import manufactured_problem
    bp = MultiphaseBlockPreconditioner(n, xi, etan, etas)
    world = dist.get_world_size(group)
    if world > 1:   # rank-local: this rank's rows of A only
        part = RowPartition(n, world, dist.get_rank(group))
        rows = torch.from_numpy(part.owned_rows(5).astype(np.int32)).cuda()
        dA = DistributedMatrix(bp.assemble_rows(_lib.OP_A, rows, c=c, d_u=d), n, 5, group=group, owned_rows=True,
                               halo=pc_kw.get("halo", "auto"))
    else:
        dA = DistributedMatrix(bp.get_big_A_matrix(c=c, d_u=d)[0], n, 5, group=group, self_halo=self_halo,
                               halo=pc_kw.get("halo", "auto"))
    del bp
    torch.cuda.empty_cache()
    M = None
    try:
        M = DistributedSchurPreconditioner(n, xi, etan, etas, c=c, d_u=d, inner_F=inner_F, inner_P=inner_P,
                                           group=group, self_halo=self_halo, **pc_kw)
        if b_vec is None:
            _, b_vec = manufactured_problem(n, c, d, xi, etan, etas)
        rows = dA.local_to_global_rows()
        assert np.array_equal(rows, M.local_to_global_rows())
        b = torch.from_numpy(np.ascontiguousarray(np.asarray(b_vec, dtype=np.float64)[rows])).cuda()
        kgroup = (group if group is not None else dist.group.WORLD) if world > 1 else None
        hist = []
        x, info = fgmres(dA, b, M=M, tol=tol, maxiter=maxiter, restrt=restrt, residuals=hist, group=kgroup)
        torch.cuda.synchronize()
    finally:
        if not keep_operators:
            dA.close()
            if M is not None:
                M.close()
    return {"x_local": x, "rows": rows, "info": info, "residuals": hist, "A": dA, "M": M}
