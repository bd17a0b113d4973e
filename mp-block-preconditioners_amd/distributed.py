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
from .csr import DeviceCSR
from .solve import PlanProfiling, _capture, _pg_stencil

N_VEL_FIELDS = 4
N_P_FIELDS = 1


@dataclass
class RowPartition:
    n: int
    world: int
    rank: int
    ghosts: bool = False   # ghost slots even at world = 1 (the periodic self-exchange; tests the halo path)

    def __post_init__(self):
        self.ghosts = self.ghosts or self.world > 1
        base, rem = divmod(self.n, self.world)
        self.r0 = self.rank * base + min(self.rank, rem)
        self.L = base + (1 if self.rank < rem else 0)
        self.r1 = self.r0 + self.L
        self.min_rows = base

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

    def __init__(self, part: RowPartition, h_u: int, h_p: int, group=None, overlap: bool = False):
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
        check(lib().mpbp_halo_set_mode(self.handle, _lib.HALO_OVERLAP if overlap else _lib.HALO_IN_ORDER))
        self.overlap = overlap
        self.fn = _lib.HALO_FN(ctypes.cast(lib().mpbp_halo_exchange, ctypes.c_void_p).value)
        self.pair_fn = _lib.HALO_PAIR_FN(ctypes.cast(lib().mpbp_halo_exchange_pair, ctypes.c_void_p).value)

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


class DistributedSchurPreconditioner(PlanProfiling):
    """The approximate-commutator apply over a row partition of the grid (one rank per GPU).

    Every rank assembles the global operators in its own HBM (setup only), keeps its rows with
    columns renumbered into the owned+ghost layout, and runs ``mpbp_schur_apply`` with halo
    callbacks; v and the result hold the rank's owned unknowns [u_n, v_n, u_s, v_s, p] rows r0..r1.
    """

    def __init__(self, n, xi, eta_n, eta_s, c=1.0, d_u=-1.0, inner_F=None, inner_P=None, group=None,
                 device=None, layout="sell", f_mode="auto", pg_mode="auto", halo="auto", self_halo=False,
                 halo_overlap=False, ca="auto", fuse_g=True):
        import torch.distributed as dist
        from .preconditioner import MultiphaseBlockPreconditioner
        from .solve import InnerSolver
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
        _, _, F, D, G = bp.get_big_A_matrix(c=c, d_u=d_u)
        GtG, GtFG = bp.commutator_products(F, D, G)
        if f_mode not in ("auto", "stencil", "assembled"):
            raise ValueError("f_mode must be 'auto', 'stencil' or 'assembled'")
        if f_mode == "stencil" and F.stencil is None:
            raise ValueError("f_mode='stencil' needs n >= 3")
        self.f_stencil = F.stencil if f_mode in ("auto", "stencil") else None
        self.pg_stencil = _pg_stencil(D, G, GtG, self.f_stencil, pg_mode)
        # inner-solver bounds from the global operators: identical on every rank
        self.inner_F = (inner_F or InnerSolver()).resolve(F, F.diagonal())
        self.inner_P = (inner_P or InnerSolver()).resolve(GtG, GtG.diagonal())
        rows_u = torch.from_numpy(part.owned_rows(N_VEL_FIELDS).astype(np.int32)).to(dev)
        rows_p = torch.from_numpy(part.owned_rows(N_P_FIELDS).astype(np.int32)).to(dev)

        def reach(M, rows):
            sub = M.extract(rows, torch.arange(M.shape[1], dtype=torch.int32, device=dev), M.shape[1])
            return halo_reach(sub.row_ptr, sub.col_idx, rows, n)

        q = reach(GtFG, rows_p)
        self.h_u = max(1, reach(F, rows_u), reach(D, rows_p))
        self.h_p = max(1, reach(G, rows_u), reach(GtG, rows_p), q)
        # communication-avoiding schedule (mpbp_schur_plan.ca): v's halo and x_b's halo only, deep enough for
        # every matrix-free operator to also compute the ghost rows its successors read
        if ca not in ("auto", True, False):
            raise ValueError("ca must be 'auto', True or False")
        self.ca, self.ca_q = False, q
        if ca and part.ghosts and self.f_stencil is not None and self.pg_stencil is not None:
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
            diag_F_glob, diag_P_glob = F.diagonal(), GtG.diagonal()
        self.F = F.extract(rows_u, cm_u, nu_ext)
        self.D = D.extract(rows_p, cm_u, nu_ext)
        self.G = G.extract(rows_u, cm_p, np_ext)
        self.GtG = GtG.extract(rows_p, cm_p, np_ext)
        self.GtFG = GtFG.extract(rows_p, cm_p, np_ext)
        del F, D, G, GtG, GtFG, bp
        torch.cuda.empty_cache()
        self.nu, self.np, self.nu_ext, self.np_ext = nu, np_, nu_ext, np_ext
        self.shape = (nu + np_, nu + np_)
        self.diag_F = self.F.diagonal()
        self.diag_P = self.GtG.diagonal()
        if self.ca:   # diagonals on owned + ghost rows (the CA schedule's ghost-row sweeps stage x0 = b / diag)
            gu = torch.from_numpy(part.ext_rows(N_VEL_FIELDS, self.h_u)).to(dev)
            gp = torch.from_numpy(part.ext_rows(N_P_FIELDS, self.h_p)).to(dev)
            self.diag_F_ext = diag_F_glob[gu].contiguous()
            self.diag_P_ext = diag_P_glob[gp].contiguous()
            del diag_F_glob, diag_P_glob

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
        f64 = dict(dtype=torch.float64, device=dev)
        self._wu = [torch.zeros(nu_ext, **f64) for _ in range(4)]
        self._wu_owned = torch.zeros(nu, **f64)
        self._wp = [torch.zeros(np_ext, **f64) for _ in range(7)]
        self._wu_ext = torch.zeros(nu_ext if self.ca else 0, **f64)
        self._tensors = {t.data_ptr(): t for t in self._wu + self._wp + ([self._wu_ext] if self.ca else [])}
        self._rccl = None
        if not self.partitioned:
            self._cb = _lib.HALO_FN()
        elif self.halo_impl == "rccl":
            self._rccl = RcclHalo(part, self.h_u, self.h_p, group, overlap=halo_overlap)
            self._cb = self._rccl.fn
        else:
            self._ex = {_lib.VEC_VELOCITY: HaloExchanger(part, N_VEL_FIELDS, self.h_u, dev, group),
                        _lib.VEC_PRESSURE: HaloExchanger(part, N_P_FIELDS, self.h_p, dev, group)}
            self._cb = _lib.HALO_FN(self._halo)
        self._prof = None
        self._plan = self._make_plan(world)

    def _halo(self, ctx, kind, x_ptr, phase, stream):
        x = self._tensors[int(x_ptr)]
        ex = self._ex[int(kind)]
        if phase == _lib.HALO_BEGIN:
            ex.begin(x)
        else:
            ex.end(x)

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
        # the in-order RCCL schedule gains nothing from splitting rows around the exchange: exchange first,
        # then one launch per sweep
        p.halo_first = 1 if (self._rccl is not None and not self._rccl.overlap) else 0
        p.ca, p.ca_reach_q = (1 if self.ca else 0), self.ca_q
        p.fuse_g = 1 if self.fuse_g else 0
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
        if self._rccl is not None:
            self._rccl.check()
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
