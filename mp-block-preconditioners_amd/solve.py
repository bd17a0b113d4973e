"""The preconditioned solve -- the reference's solve.py surface, with the apply on the GPU.

    ApproxSchurPreconditioner  ~ approx_schur = LinearOperator(matvec=approx_schur_op)  solve.py:240-281
    fgmres                     ~ pyamg.krylov.fgmres (the outer Krylov loop)           solve.py:285
    solve_with_approx_schur_pc ~ solve.py:240-286
    Jacobi                     ~ solve.py:149-159 (as an inner solver kind)

The reference factors F and Gt_G with ilupp's ILUT (solve.py:251-254; sequential triangular
solves).  On MI355X the inner inverses are the fused Jacobi / Chebyshev-Jacobi SpMV sweeps of
libmpbp (``InnerSolver``); the outer composition of approx_schur_op is unchanged and runs as one
native call (``mpbp_schur_apply``) that is graph-capturable.
"""
from __future__ import annotations

import ctypes
import os
import math
from dataclasses import dataclass

import numpy as np
import scipy.sparse.linalg as spla
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_handle
from .csr import DeviceCSR
from .preconditioner import MultiphaseBlockPreconditioner, PGStencil


@dataclass
class InnerSolver:
    """Approximate inverse used for F^-1 and Gt_G^-1 inside the apply.

    kind   "jacobi" (solve.py:149-159), "chebyshev" (Chebyshev-Jacobi, BASELINE configs[3]) or "mg" (geometric
           multigrid V-cycles, the reference's pointer at solve.py:266/274; mg.Multigrid)
    sweeps updates of x from x0 = 0 (sweeps - 1 SpMVs); for "mg" the number of V-cycles
    lmax   upper bound of spec(diag(M)^-1 M); None -> Gershgorin bound computed on the GPU
    lmin   lower end of the Chebyshev interval; None -> lmax / ratio
    pre, post, smooth_ratio, coarsest   "mg" only: smoothing sweeps per level, smoothing interval
           [lmax / smooth_ratio, lmax], coarsening stops at n <= coarsest
    """
    kind: str = "chebyshev"
    sweeps: int = 4
    lmin: float | None = None
    lmax: float | None = None
    ratio: float = 30.0
    pre: int = 2
    post: int = 2
    smooth_ratio: float = 4.0
    coarsest: int = 16     # dense coarsest inverse at 16^2: 1024 x 1024 for F (one fewer latency-bound level than 8^2)

    def resolve(self, M: DeviceCSR, diag: torch.Tensor) -> "InnerSolver":
        if self.kind == "jacobi":
            return InnerSolver("jacobi", int(self.sweeps), 0.0, 0.0, self.ratio)
        if self.kind == "mg":
            return InnerSolver("mg", int(self.sweeps), 0.0, 0.0, self.ratio, int(self.pre), int(self.post),
                               float(self.smooth_ratio), int(self.coarsest))
        if self.kind != "chebyshev":
            raise ValueError(f"unknown inner solver {self.kind!r}")
        lmax = float(self.lmax) if self.lmax is not None else M.gershgorin(diag)
        lmin = float(self.lmin) if self.lmin is not None else lmax / self.ratio
        return InnerSolver("chebyshev", int(self.sweeps), lmin, lmax, self.ratio)

    def multigrid(self, M: DeviceCSR, n: int, fields, diag: torch.Tensor):
        from .mg import Multigrid
        return Multigrid(M, n, fields, pre=self.pre, post=self.post, cycles=int(self.sweeps),
                         ratio=self.smooth_ratio, coarsest=self.coarsest, diag=diag, fine_sell=False)

    def cstruct(self):
        kind = {"chebyshev": _lib.INNER_CHEBYSHEV, "jacobi": _lib.INNER_JACOBI, "mg": _lib.INNER_MG}[self.kind]
        return _lib.InnerSolverC(kind, int(self.sweeps), float(self.lmin or 0.0), float(self.lmax or 0.0))


NUMERICS = ("exact", "fast")


def _check_numerics(numerics: str) -> str:
    """'exact': the matrix-free F sweeps perform the assembly's IEEE operations in CSR order (bit-identical to the
    sequential oracle); 'fast': the same operator regrouped per coefficient and FMA-contracted with reciprocal diagonals
    (MPBP_NUMERICS_FAST), north_star's bar -- within 1e-12 relative inf-norm of the oracle apply.  What 'fast'
    changes: the matrix-free F rows (inner solves, multigrid level-0 smoothing and residuals); on one GPU Gt_F_G x from
    the diamond's symmetric half (kernel option q13_sym, kept only when the stored product is symmetric to 1e-14); and
    the multigrid hierarchies' level 1 applied matrix-free as R0 (F (P0 x)) / R0 (Gt_G (P0 x)) (kernel options
    mg_galerkin_mf / mg_galerkin_mf_p).  D, G, Gt_G and the other kernels compute the same bits in both modes."""
    if numerics not in NUMERICS:
        raise ValueError(f"numerics must be one of {NUMERICS}")
    return numerics


def _device_csr(M, device):
    return M if isinstance(M, DeviceCSR) else DeviceCSR.from_scipy(M, device)


def event_device_scope() -> int:
    """1 (default): profiling events release at device scope (mpbp_event_create_scoped), so recording one between two
    sweeps does not write the L2 back to HBM and the timed sweep runs as it does inside the captured apply;
    MPBP_EVENT_SCOPE=system restores hipEventDefault."""
    return 0 if os.environ.get("MPBP_EVENT_SCOPE", "device") == "system" else 1


class DeviceEvent:
    """A timing hipEvent from libmpbp (device-scope release by default, event_device_scope)."""

    def __init__(self):
        self.h = ctypes.c_void_p()
        check(lib().mpbp_event_create_scoped(ctypes.byref(self.h), event_device_scope()))

    def record(self, stream=None):
        check(lib().mpbp_event_record(self.h, stream if stream is not None else stream_handle()))

    def elapsed_ms(self, end: "DeviceEvent") -> float:
        ms = ctypes.c_float(0.0)
        check(lib().mpbp_event_elapsed_ms(self.h, end.h, ctypes.byref(ms)))
        return ms.value

    def __del__(self):
        try:
            if self.h:
                lib().mpbp_event_destroy(self.h)
        except Exception:
            pass


class PlanProfiling:
    """What the Schur preconditioners share around their mpbp_schur_plan: the plan's kernel choices
    (set_kernel_opts) and hipEvent pairs recorded by mpbp_schur_apply around every inner-F SpMV sweep (bench.py)."""

    def set_kernel_opts(self, **kw):
        """Change this preconditioner's kernel choices (mpbp_kernel_opts field names; others untouched).  The next apply
        or capture uses them; graphs captured before keep the choices they were captured with.  Every choice computes
        the same bits except q13_sym, q13_mf and mg_coarse_tree (tolerance mode; q13_sym stays 0 where the stored Gt_F_G
        is not symmetric, q13_mf where it is not the product of the preconditioner's own F, D, G)."""
        names = {f for f, _ in _lib.KernelOpts._fields_ if f != "reserved"}
        for k, v in kw.items():
            if k not in names:
                raise ValueError(f"unknown kernel option {k!r} (known: {sorted(names)})")
            if k == "q13_mf" and v and not getattr(self, "gtfg_is_product", False):
                raise ValueError("q13_mf: this preconditioner's Gt_F_G is not known to be ((-D) F) G of its own "
                                 "F, D, G (pass GtFG from commutator_products of the same operators, or none)")
            if k == "q13_sym" and v and getattr(self, "q13_asymmetry", None) is not None:
                a, m = self.q13_asymmetry
                if not a <= 1e-14 * m:
                    raise ValueError(f"q13_sym: this Gt_F_G is not symmetric (max |Q - Q^T| {a:.3g}, max |Q| {m:.3g})")
            setattr(self.kernel_opts, k, int(v))

    def enable_profiling(self, capacity: int):
        evs = (ctypes.c_void_p * (2 * capacity))()
        for i in range(2 * capacity):
            e = ctypes.c_void_p()
            check(lib().mpbp_event_create_scoped(ctypes.byref(e), event_device_scope()))
            evs[i] = e
        cnt = ctypes.c_int32(0)
        self._prof = (evs, cnt, capacity)
        self._plan.prof_events = ctypes.cast(evs, ctypes.c_void_p)
        self._plan.prof_capacity = capacity
        self._plan.prof_count = ctypes.pointer(cnt)

    def reset_profiling(self):
        if self._prof:
            self._prof[1].value = 0

    def profiled_ms(self):
        """Durations (ms) of the recorded inner-F sweeps (call after synchronising)."""
        if not self._prof:
            return []
        evs, cnt, _ = self._prof
        out = []
        for i in range(cnt.value):
            ms = ctypes.c_float(0.0)
            check(lib().mpbp_event_elapsed_ms(evs[2 * i], evs[2 * i + 1], ctypes.byref(ms)))
            out.append(ms.value)
        return out

    def disable_profiling(self):
        if self._prof:
            evs, _, cap = self._prof
            for i in range(2 * cap):
                lib().mpbp_event_destroy(evs[i])
        self._prof = None
        self._plan.prof_events = None
        self._plan.prof_capacity = 0
        self._plan.prof_count = ctypes.POINTER(ctypes.c_int32)()


def _pg_stencil(D, G, GtG, f_stencil, pg_mode):
    """The PGStencil of Gt_G when D, G and Gt_G can run matrix-free (pg_mode 'auto' / 'stencil'), else None."""
    if pg_mode not in ("auto", "stencil", "assembled"):
        raise ValueError("pg_mode must be 'auto', 'stencil' or 'assembled'")
    if pg_mode == "assembled":
        return None
    sd, sg, sp = (getattr(M, "stencil", None) for M in (D, G, GtG))
    ok = all(isinstance(s, PGStencil) for s in (sd, sg, sp)) and \
        (sd.op, sg.op, sp.op) == (_lib.PG_D, _lib.PG_G, _lib.PG_GTG) and sd.same_grid(sg) and sd.same_grid(sp) and \
        (f_stencil is None or sd.same_grid(f_stencil))
    if not ok and pg_mode == "stencil":
        raise ValueError("pg_mode='stencil' needs D, G from one get_big_A_matrix call (n >= 3) and Gt_G from "
                         "commutator_products")
    return sp if ok else None


def _q13_layout(Q: DeviceCSR, q_mode: str):
    """(n, values[13 n^2]) of Gt_F_G in the diamond layout (mpbp_q13_build), or None (q_mode 'assembled', or
    'auto' on an operator that is not the 13-point periodic-grid product)."""
    if q_mode not in ("auto", "diamond", "assembled"):
        raise ValueError("q_mode must be 'auto', 'diamond' or 'assembled'")
    if q_mode == "assembled":
        return None
    n = math.isqrt(Q.shape[0])
    if n * n != Q.shape[0] or Q.shape != (n * n, n * n) or n < 5:
        if q_mode == "diamond":
            raise ValueError("q_mode='diamond' needs Gt_F_G of an n x n grid, n >= 5")
        return None
    vals = torch.empty(13 * n * n, dtype=torch.float64, device=Q.device)
    rc = lib().mpbp_q13_build(ctypes.byref(Q.cstruct()), n, ptr(vals), stream_handle())
    if rc:
        if q_mode == "diamond":
            raise ValueError(f"q_mode='diamond': {lib().mpbp_last_error().decode()}")
        return None
    return n, vals


def _capture(pc, v: torch.Tensor, out: torch.Tensor, capture_error_mode: str = "global"):
    """One pc.apply(v, out) captured into a torch.cuda.CUDAGraph (warm-up on a side stream first).
    capture_error_mode "thread_local" lets other threads (RCCL's proxy thread) keep making HIP calls that
    are illegal during a global-mode capture."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    saved = (pc._plan.prof_events, pc._plan.prof_capacity)
    pc._plan.prof_events, pc._plan.prof_capacity = None, 0
    try:
        with torch.cuda.stream(s):
            pc.apply(v, out)                    # warm-up on a side stream, as torch requires
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode=capture_error_mode):
            pc.apply(v, out)
    finally:
        pc._plan.prof_events, pc._plan.prof_capacity = saved
    return g


class ApproxSchurPreconditioner(PlanProfiling, spla.LinearOperator):
    """M^-1 of the block upper-triangular approximate-commutator preconditioner (solve.py:257-277).

    ``apply(v, out)`` works on CUDA tensors and is graph-capturable; ``matvec`` (the scipy
    LinearOperator surface) copies a host vector in and out around the same apply.
    """

    def __init__(self, F, D, G, GtG=None, GtFG=None, inner_F: InnerSolver | None = None,
                 inner_P: InnerSolver | None = None, device=None, layout: str = "sell", f_mode: str = "auto",
                 pg_mode: str = "auto", q_mode: str = "auto", fuse_g: bool = True, numerics: str = "exact",
                 kernel_opts: dict | None = None):
        dev = torch.device(device or (F.device if isinstance(F, DeviceCSR) else "cuda"))
        self.numerics = _check_numerics(numerics)
        # this preconditioner's kernel choices (mpbp_kernel_opts): the process defaults now, with `kernel_opts`
        # overrides -- later mpbp_set_* calls and other preconditioners' choices do not affect it
        self.kernel_opts = _lib.kernel_opts(kernel_opts)
        self.F, self.D, self.G = (_device_csr(M, dev) for M in (F, D, G))
        if GtG is None or GtFG is None:
            GtG, GtFG = MultiphaseBlockPreconditioner.commutator_products(self.F, self.D, self.G)
        self.GtG, self.GtFG = _device_csr(GtG, dev), _device_csr(GtFG, dev)
        # Gt_F_G is the product of this preconditioner's own F, D, G (commutator_products of these objects): only then
        # may tolerance mode apply it matrix-free as -(D (F (G x))) (kernel option q13_mf)
        tag = getattr(self.GtFG, "_product_of", None)
        self.gtfg_is_product = tag is not None and all(r() is M for r, M in zip(tag, (self.F, self.D, self.G)))
        if not self.gtfg_is_product:
            self.kernel_opts.q13_mf = 0
        nu, np_ = self.F.shape[0], self.GtG.shape[0]
        if self.F.shape != (nu, nu) or self.D.shape != (np_, nu) or self.G.shape != (nu, np_) \
                or self.GtFG.shape != (np_, np_):
            raise ValueError("inconsistent block shapes")
        self.nu, self.np = nu, np_
        self.device = dev
        self.diag_F = self.F.diagonal()
        self.diag_P = self.GtG.diagonal()
        self.inner_F = (inner_F or InnerSolver()).resolve(self.F, self.diag_F)
        self.inner_P = (inner_P or InnerSolver()).resolve(self.GtG, self.diag_P)
        # multigrid inner solves: hierarchies over F (4 velocity fields) and Gt_G (pressure) of the n x n grid
        self.mg_F = self.mg_P = None
        if "mg" in (self.inner_F.kind, self.inner_P.kind):
            from .mg import FIELDS_PRESSURE, FIELDS_VELOCITY
            n = math.isqrt(np_)
            if n * n != np_ or nu != 4 * np_:
                raise ValueError("multigrid inner solves need the n x n MAC-grid operators")
            if self.inner_F.kind == "mg":
                self.mg_F = self.inner_F.multigrid(self.F, n, FIELDS_VELOCITY, self.diag_F)
            if self.inner_P.kind == "mg":
                self.mg_P = self.inner_P.multigrid(self.GtG, n, FIELDS_PRESSURE, self.diag_P)
        f64 = dict(dtype=torch.float64, device=dev)
        self._wu = [torch.empty(nu, **f64) for _ in range(4)]
        self._wu_owned = torch.empty(nu, **f64)
        self._wp = [torch.empty(np_, **f64) for _ in range(7)]
        self._prof = None
        if layout not in ("sell", "csr"):
            raise ValueError("layout must be 'sell' or 'csr'")
        self.layout = layout
        self._sell = [M.to_sell() for M in (self.F, self.D, self.G, self.GtG, self.GtFG)] if layout == "sell" else None
        # F sweeps: "stencil" recomputes F's rows from thn (bit-identical to the assembled F, ~4x fewer
        # HBM bytes); "assembled" streams the stored F; "auto" = stencil whenever F carries one.
        if f_mode not in ("auto", "stencil", "assembled"):
            raise ValueError("f_mode must be 'auto', 'stencil' or 'assembled'")
        st = getattr(self.F, "stencil", None)
        if f_mode == "stencil" and st is None:
            raise ValueError("f_mode='stencil' needs F from MultiphaseBlockPreconditioner.get_big_A_matrix (n >= 3)")
        self.f_stencil = st if f_mode in ("auto", "stencil") else None
        # D, G, Gt_G likewise ("pg"): recomputed from the cell thn table when all three carry stencils of
        # one grid (get_big_A_matrix + commutator_products), else streamed from their stored copies.
        self.pg_stencil = _pg_stencil(self.D, self.G, self.GtG, self.f_stencil, pg_mode)
        # Gt_F_G: "diamond" streams its values in the 13-point diamond layout (columns implicit in the grid,
        # 104 B per row instead of 156), "assembled" the CSR / SELL copy; "auto" = diamond whenever Gt_F_G is
        # the n^2 x n^2 periodic-grid product (n >= 5), else assembled.
        self.q13 = _q13_layout(self.GtFG, q_mode)
        # tolerance mode reads Gt_F_G's symmetric half only when the stored product IS symmetric (to 1e-14 of its
        # largest entry; G^T F G is, to rounding) -- a caller's non-symmetric Gt_F_G keeps all 13 slots
        self.q13_asymmetry = None
        if self.q13 is not None and self.numerics == "fast":
            a = (ctypes.c_double * 2)()
            check(lib().mpbp_q13_asymmetry(self.q13[0], ptr(self.q13[1]), a, stream_handle()))
            self.q13_asymmetry = (a[0], a[1])
            if not a[0] <= 1e-14 * a[1]:
                self.kernel_opts.q13_sym = 0
        # the second F solve recomputes its right-hand side G x_p inside its sweeps (no G launch, W never stored)
        # when F and G are both matrix-free and F's inner solve is Chebyshev with >= 2 sweeps; same bits
        self.fuse_g = bool(fuse_g and self.f_stencil is not None and self.pg_stencil is not None
                           and self.inner_F.kind == "chebyshev" and self.inner_F.sweeps >= 2)
        self._plan = self._make_plan()
        super().__init__(dtype=np.float64, shape=(nu + np_, nu + np_))

    def _make_plan(self):
        p = _lib.SchurPlan()
        p.nu, p.np, p.nu_ext, p.np_ext = self.nu, self.np, self.nu, self.np
        p.F, p.D, p.G = self.F.cstruct(), self.D.cstruct(), self.G.cstruct()
        p.GtG, p.GtFG = self.GtG.cstruct(), self.GtFG.cstruct()
        empty = _lib.RowBlocks(None, 0)
        p.F_int, p.F_bnd = self.F.blocks.cstruct(), empty
        p.D_int, p.D_bnd = self.D.blocks.cstruct(), empty
        p.G_int, p.G_bnd = self.G.blocks.cstruct(), empty
        p.P_int, p.P_bnd = self.GtG.blocks.cstruct(), empty
        p.Q_int, p.Q_bnd = self.GtFG.blocks.cstruct(), empty
        p.diag_F, p.diag_P = self.diag_F.data_ptr(), self.diag_P.data_ptr()
        p.inner_F, p.inner_P = self.inner_F.cstruct(), self.inner_P.cstruct()
        for i, t in enumerate(self._wu):
            p.wu[i] = t.data_ptr()
        p.wu_owned = self._wu_owned.data_ptr()
        for i, t in enumerate(self._wp):
            p.wp[i] = t.data_ptr()
        p.use_sell = 1 if self._sell else 0
        if self._sell:
            esell = _lib.Sell(0, 0, 0, 0, None, None, None, None)
            for name, S in zip(("Fs", "Ds", "Gs", "Ps", "Qs"), self._sell):
                setattr(p, name + "_int", S.cstruct())
                setattr(p, name + "_bnd", esell)
        p.f_stencil = 1 if self.f_stencil is not None else 0
        if self.f_stencil is not None:
            p.f_prm = self.f_stencil.prm
            p.f_cell, p.f_uface, p.f_vface = (t.data_ptr() for t in (self.f_stencil.cell, self.f_stencil.uface,
                                                                    self.f_stencil.vface))
        p.pg_stencil = 1 if self.pg_stencil is not None else 0
        if self.pg_stencil is not None and self.f_stencil is None:
            p.f_prm, p.f_cell = self.pg_stencil.prm, self.pg_stencil.cell.data_ptr()
        p.halo = _lib.HALO_FN()
        p.halo_ctx = None
        p.prof_events = None
        p.prof_capacity = 0
        p.prof_count = ctypes.POINTER(ctypes.c_int32)()
        if self.q13 is not None:
            p.q13, p.q13_n = self.q13[1].data_ptr(), self.q13[0]
        if self.mg_F is not None:
            p.mg_F = ctypes.pointer(self.mg_F.cstruct())
        if self.mg_P is not None:
            p.mg_P = ctypes.pointer(self.mg_P.cstruct())
        p.fuse_g = 1 if self.fuse_g else 0
        p.f_numerics = _lib.NUMERICS_FAST if self.numerics == "fast" else _lib.NUMERICS_EXACT
        p.opts = ctypes.pointer(self.kernel_opts)
        return p

    def sell_of(self, key):
        """The SELL-64 copy of F / D / G / P (Gt_G) / Q (Gt_F_G), or None in the CSR layout."""
        return self._sell["FDGPQ".index(key)] if self._sell else None

    # -- the apply ---------------------------------------------------------------------------------
    def apply(self, v: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        assert v.is_cuda and v.dtype == torch.float64 and v.numel() == self.nu + self.np
        if out is None:
            out = torch.empty_like(v)
        check(lib().mpbp_schur_apply(ctypes.byref(self._plan), ptr(v), ptr(out), stream_handle()))
        return out

    def capture(self, v: torch.Tensor, out: torch.Tensor):
        """Capture one apply(v, out) into a hipGraph (torch.cuda.CUDAGraph); replay() re-runs it on the
        same buffers.  mpbp_schur_apply allocates and synchronises nothing, so the whole apply becomes
        one graph launch (profiling events are recorded by eager applies only)."""
        return _capture(self, v, out)

    def _matvec(self, x):
        """Host vector in, host vector out (the LinearOperator surface pyamg drives, solve.py:281): staged
        through page-locked buffers allocated on first use, so both PCIe copies run at DMA speed.  One call
        at a time per preconditioner (the staging buffers are shared; a lock serialises threads)."""
        return _staged_host_call(self, x, self.nu + self.np, self.nu + self.np, self.device, self.apply)

    def release_staging(self):
        """Free the page-locked / device staging buffers of the host-vector matvec (re-created on demand)."""
        self._pinned = None

    # reference naming (solve.py:257)
    def approx_schur_op(self, v):
        return self._matvec(v)


def _staged_host_call(obj, x, n_in, n_out, device, fn):
    """y = fn(x_dev, y_dev) for a host vector x of n_in entries through obj's page-locked staging buffers.
    Raises like scipy on a wrong length (no broadcasting); the stream is synchronised even when fn raises,
    so the next call never overwrites a buffer a DMA is still reading."""
    import threading
    x = np.ravel(np.asarray(x))
    if x.shape != (n_in,):
        raise ValueError(f"dimension mismatch: operand has {x.shape[0]} entries, the operator takes {n_in}")
    lock = obj.__dict__.setdefault("_stage_lock", threading.Lock())
    with lock:
        if getattr(obj, "_pinned", None) is None:
            obj._pinned = (torch.empty(n_in, dtype=torch.float64, pin_memory=True),
                           torch.empty(n_out, dtype=torch.float64, pin_memory=True),
                           torch.empty(n_in, dtype=torch.float64, device=device),
                           torch.empty(n_out, dtype=torch.float64, device=device))
        h_in, h_out, d_in, d_out = obj._pinned
        stream = torch.cuda.current_stream(device)
        try:
            h_in.numpy()[:] = x
            d_in.copy_(h_in, non_blocking=True)
            fn(d_in, d_out)
            h_out.copy_(d_out, non_blocking=True)
        finally:
            stream.synchronize()
        return h_out.numpy().copy()


def _as_operator(A):
    if A is None:
        return None
    if isinstance(A, DeviceCSR):
        return lambda x, out=None: A.matvec(x, out=out)
    if hasattr(A, "apply"):   # ApproxSchurPreconditioner, DistributedSchurPreconditioner, DistributedMatrix
        return lambda x, out=None: A.apply(x, out=out)
    if callable(A):
        return lambda x, out=None: A(x)
    raise TypeError(f"unsupported operator {type(A)}")


def _apply_into(op, x, w):
    """w = op(x) in fgmres's own buffer: operators that take `out` write it there (no 42 MB copy per iteration at
    1024^2); a result elsewhere (an operator without `out`) is copied in -- the caller's tensor is never modified."""
    y = op(x, out=w)
    if y is not w:
        w.copy_(y)


_KCHUNK = 256   # basis vectors per mpbp_rdot / mpbp_gs_update launch


class KrylovKernels:
    """FGMRES's vector kernels on CUDA float64 vectors through libmpbp, optionally over the ranks of a row partition.

    Inner products are reproducible (``mpbp_rdot``: binned sums whose fold sums add exactly, so the result depends only
    on the set of terms); their bounds are max-reductions and their fold sums sum-reductions over ``group``.  Every other
    step is element-wise in a fixed order (``mpbp_gs_update``).  FGMRES therefore computes the same bits on one GPU and
    on any row partition whose operator and preconditioner applies are bit-exact (DistributedMatrix,
    DistributedSchurPreconditioner): same residual history, same iterate."""

    def __init__(self, n: int, kmax: int, device, group=None):
        self.n, self.group, self.kmax = int(n), group, int(kmax)
        self.device = torch.device(device)
        self.backend = None
        n_total = self.n
        if group is not None:
            import torch.distributed as dist
            self.dist = dist
            self.backend = dist.get_backend(group)
            t = torch.tensor([self.n], dtype=torch.int64)
            t = self._reduce(t.to(self.device) if self.backend == "nccl" else t, "sum")
            n_total = int(t.item())
        self.n_total = n_total
        f64 = dict(dtype=torch.float64, device=self.device)
        self.part = torch.empty(max(1, int(lib().mpbp_rdot_part_size(self.n, min(self.kmax, _KCHUNK)))), **f64)
        self.acc = torch.empty(3 * self.kmax, **f64)
        self.h = torch.empty(self.kmax, **f64)

    def _reduce(self, t: torch.Tensor, op: str) -> torch.Tensor:
        if self.group is None:
            return t
        rop = self.dist.ReduceOp.SUM if op == "sum" else self.dist.ReduceOp.MAX
        if self.backend == "nccl" or t.device.type == "cpu":
            self.dist.all_reduce(t, op=rop, group=self.group)
            return t
        c = t.cpu()   # gloo: host-staged
        self.dist.all_reduce(c, op=rop, group=self.group)
        t.copy_(c)
        return t

    def amax(self, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """out[0] = max |x| over every rank."""
        check(lib().mpbp_absmax(ptr(x), x.numel(), ptr(out), stream_handle()))
        return self._reduce(out, "max")

    def fold_sums(self, V: torch.Tensor, ld: int, k: int, w: torch.Tensor, vb: torch.Tensor, wb: torch.Tensor):
        """acc[:3k]: the exact fold sums of V[i] . w over every rank (basis rows in chunks of 256 per launch)."""
        for i0 in range(0, k, _KCHUNK):
            kc = min(_KCHUNK, k - i0)
            check(lib().mpbp_rdot(ctypes.c_void_p(V.data_ptr() + 8 * i0 * ld), ld, kc, ptr(w), self.n, self.n_total,
                                  ctypes.c_void_p(vb.data_ptr() + 8 * i0), ptr(wb), ptr(self.part),
                                  ctypes.c_void_p(self.acc.data_ptr() + 24 * i0), stream_handle()))
        return self._reduce(self.acc[: 3 * k], "sum")

    def dots(self, V, ld, k, w, vb, wb) -> torch.Tensor:
        """h[:k] = V[:k] w (device)."""
        self.fold_sums(V, ld, k, w, vb, wb)
        check(lib().mpbp_rdot_finish(k, ptr(self.acc), ptr(self.h), stream_handle()))
        return self.h[:k]

    def update_dots(self, V, ld, k, h, w, vb, wb) -> torch.Tensor:
        """CGS2's first update and second projection in one pass over V[:k] (k <= 256): w <- w - V[:k]^T h in place
        (``update``'s bits), then h2 = V[:k] w, its fold extractors from the a-priori bound wb[0] + sum vb |h| (wb[0]:
        max |w| before the update, over every rank) -- reproducible over any row partition like ``dots``."""
        check(lib().mpbp_gs_update_rdot(ptr(V), ld, k, ptr(h), ptr(w), self.n, self.n_total, ptr(vb), ptr(wb), ptr(w),
                                         ptr(self.part), ptr(self.acc), stream_handle()))
        self._reduce(self.acc[: 3 * k], "sum")
        check(lib().mpbp_rdot_finish(k, ptr(self.acc), ptr(self.h), stream_handle()))
        return self.h[:k]

    # -- DCGS2 (two basis passes per iteration; fgmres(ortho="dcgs2")) --------------------------------------------------
    def block_folds(self, V, ld, k, u, w, vb, bu, bw) -> torch.Tensor:
        """The exact fold sums of V[:k] . u and V[:k] . w in one pass over V (k <= 256), summed over every rank:
        acc2[:3k] for u, acc2[3k:6k] for w (mpbp_rdot2)."""
        if not hasattr(self, "acc2"):
            f64 = dict(dtype=torch.float64, device=self.device)
            self.part2 = torch.empty(max(1, int(lib().mpbp_rdot_part_size(self.n, 2 * min(self.kmax, _KCHUNK)))), **f64)
            self.acc2 = torch.empty(6 * _KCHUNK, **f64)
            self.hu, self.hw = torch.empty(_KCHUNK, **f64), torch.empty(_KCHUNK, **f64)
            self.P = torch.empty(4, **f64)
        check(lib().mpbp_rdot2(ptr(V), ld, k, ptr(u), ptr(w), self.n, self.n_total, ptr(vb), ptr(bu), ptr(bw),
                               ptr(self.part2), ptr(self.acc2), stream_handle()))
        return self._reduce(self.acc2[: 6 * k], "sum")

    def dcgs2_update(self, V, ld, j, acc, bw, w, upd_w=True):
        """Iteration j's scalars and updates (mpbp_dcgs2_update): V[j] <- q_j, V[j+1] <- u_{j+1} (upd_w); returns the
        device tensors (hu[:j+1], hw[:j+1], P = [r, 1/r, c, bound of u_{j+1}])."""
        check(lib().mpbp_dcgs2_update(ptr(V), ld, j, ptr(acc), ptr(bw), ptr(w), self.n, 1 if upd_w else 0, ptr(self.hu),
                                      ptr(self.hw), ptr(self.P), stream_handle()))
        return self.hu[: j + 1], self.hw[: j + 1], self.P

    def update(self, V, ld, k, h, w, out):
        """out = w - V[:k]^T h (out may be w), the basis rows in chunks of 256 (a fixed order)."""
        src = w
        for i0 in range(0, k, _KCHUNK):
            kc = min(_KCHUNK, k - i0)
            check(lib().mpbp_gs_update(ctypes.c_void_p(V.data_ptr() + 8 * i0 * ld), ld, kc,
                                       ctypes.c_void_p(h.data_ptr() + 8 * i0), ptr(src), self.n, ptr(out),
                                       stream_handle()))
            src = out
        return out


def _finish(a) -> float:
    """h = (S0 + S1) + S2 from a fold-sum triple -- mpbp_rdot_finish's IEEE operations on the host."""
    return (float(a[0]) + float(a[1])) + float(a[2])


def _solve_upper(H, g, k):
    """y = triu(H[:k, :k])^-1 g[:k] by back substitution in a fixed order (host IEEE arithmetic: the same bits on
    every rank and in every process)."""
    y = [0.0] * k
    for i in range(k - 1, -1, -1):
        t = float(g[i])
        for j in range(i + 1, k):
            t -= float(H[i, j]) * y[j]
        y[i] = t / float(H[i, i])
    return y


_VB_SLACK = 1.0 + 2.0 ** -50   # |fl(w / s)| <= fl(max|w| / s) (1 + 2^-50): the new basis vector's bound


def fgmres(A, b, x0=None, tol=1e-5, restrt=None, maxiter=None, M=None, callback=None, residuals=None,
           capture_M=True, group=None, kernels=None, fused_cgs2=False, ortho="dcgs2"):
    """Flexible GMRES with right preconditioning, all vectors in HBM.

    Same call shape as pyamg.krylov.fgmres (solve.py:207, 237, 285): convergence when the
    residual 2-norm falls below ``tol * ||r0||``; returns (x, info) with info 0 on convergence
    and the iteration count otherwise.  ``callback(xk)`` receives the current iterate as a CUDA
    tensor after every inner iteration (the reference's true-residual printer, solve.py:161-170).
    Orthogonalisation (``ortho``): "dcgs2" (default) -- classical Gram-Schmidt with the re-orthogonalisation pass
    delayed into the next iteration's block product (Swirydowicz et al. 2020, Bielich et al. 2022): two sweeps over the
    basis per iteration (``mpbp_rdot2``, ``mpbp_dcgs2_update``), H's column j completed one iteration later; "cgs2" --
    two full CGS passes per iteration (four sweeps: ``mpbp_rdot`` + ``mpbp_gs_update`` twice).  Both with reproducible
    inner products (``KrylovKernels``); restarts longer than 255 take CGS2.
    pyamg is not installed here, so iteration counts against pyamg itself are unpinned.

    group: the process group of a row partition -- b, x0 and the vectors A and M take and return are the rank's
    owned rows (DistributedMatrix, DistributedSchurPreconditioner); the iterates are bit-identical to the one-GPU
    solve's rows.  kernels: a KrylovKernels-compatible object (default: libmpbp's).
    fused_cgs2: CGS2's first update and second projection in one kernel (``update_dots``; the second projection's fold
    extractors from an a-priori bound on the updated vector), meant to save one of the four passes over the basis per
    iteration.  Off by default: its re-read of the chunk's basis entries misses the caches at 1024^2 and it measured no
    faster; False: the two projections apart (max |w| measured before each).
    capture_M: an ApproxSchurPreconditioner M (or a partitioned one over the in-order RCCL halo) is captured once into
    a hipGraph and replayed per iteration (its launches -- hundreds with multigrid inner solves -- then cost one graph
    launch; the iteration's host work never starves the GPU); same results as eager applies.
    """
    Aop = _as_operator(A)
    Mop = _as_operator(M)
    b = b if isinstance(b, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(b, dtype=np.float64)).cuda()
    if kernels is None and not (b.is_cuda and b.dtype == torch.float64):
        raise TypeError("fgmres runs on CUDA float64 vectors (libmpbp kernels); there is no CPU fallback")
    n = b.numel()
    # the defaults follow the GLOBAL length (pyamg's min(n, 200) of the whole system): with a group every rank must run
    # the same iterations -- a rank-local default would let one rank leave the loop while the others still wait in the
    # inner products' all-reduces -- and the partitioned solve must stay the one-GPU solve bit for bit
    n_glob = n
    if group is not None and (maxiter is None or restrt is None):
        import torch.distributed as dist
        t = torch.tensor([n], dtype=torch.int64)
        if dist.get_backend(group) == "nccl":
            t = t.to(b.device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        n_glob = int(t.item())
    maxiter = int(maxiter) if maxiter is not None else min(n_glob, 200)
    m = int(restrt) if restrt is not None else maxiter
    if capture_M and M is not None and hasattr(M, "capture") and b.is_cuda:
        try:
            # the captured apply is kept on M and reused by later solves with the same M (capturing and instantiating
            # a multigrid apply's hundreds of launches costs tens of ms)
            cached = getattr(M, "_fgmres_graph", None)
            if cached is not None and cached[0].device == b.device:
                m_in, m_out, m_graph = cached
            else:
                m_in = torch.zeros(M.shape[0], dtype=torch.float64, device=b.device)
                m_out = torch.empty_like(m_in)
                m_graph = M.capture(m_in, m_out)
                try:
                    M._fgmres_graph = (m_in, m_out, m_graph)
                except AttributeError:
                    pass

            def Mop(x, out=None, _g=m_graph, _i=m_in, _o=m_out):   # noqa: F811
                _i.copy_(x)
                _g.replay()
                return _o
        except NotImplementedError:   # e.g. a partitioned apply over the host-staged (gloo) halo: eager
            pass
    K = kernels if kernels is not None else KrylovKernels(n, m + 1, b.device, group)
    if ortho not in ("dcgs2", "cgs2"):
        raise ValueError("ortho must be 'dcgs2' or 'cgs2'")
    if ortho == "dcgs2" and m + 1 <= 256 and hasattr(K, "block_folds") and not fused_cgs2:
        return _fgmres_dcgs2(Aop, Mop, b, x0, tol, m, maxiter, callback, residuals, K)
    fused = fused_cgs2 and hasattr(K, "update_dots")
    f64 = dict(dtype=b.dtype, device=b.device)
    x = torch.zeros_like(b) if x0 is None else (
        x0.clone() if isinstance(x0, torch.Tensor) else torch.from_numpy(np.asarray(x0, dtype=np.float64)).to(b.device))
    bnd = torch.empty(2, **f64)          # [max |r|, max |w|]

    def norm(v, slot):
        K.amax(v, bnd[slot:slot + 1])
        a = K.fold_sums(v, n, 1, v, bnd[slot:slot + 1], bnd[slot:slot + 1])
        return math.sqrt(_finish(a.cpu().tolist()))

    def lincomb(xv, Zm, k, y):
        """xv + Zm[:k]^T y (element-wise, basis vectors added in order)."""
        ny = torch.from_numpy(-np.asarray(y[:k], dtype=np.float64)).to(b.device)
        return K.update(Zm, n, k, ny, xv, torch.empty_like(xv))

    r = b - Aop(x)
    normr = norm(r, 0)
    if residuals is not None:
        residuals[:] = [normr]
    normb = norm(b, 1) or 1.0
    if normr < tol * normb:
        return x, 0
    target = tol * normr if normr != 0.0 else tol
    it = 0
    w = torch.empty_like(b)
    # the basis and the preconditioned directions are only read in the rows already written (dots, update and lincomb
    # take the first j + 1 / k rows): left uninitialised -- two (m + 1) x n memsets (7.6 GB at 1024^2) saved
    V = torch.empty(m + 1, n, **f64)
    Z = torch.empty(m, n, **f64)
    vb = torch.zeros(m + 1, **f64)       # max |V[i]| bounds (identical on every rank)
    # the iteration's scalars (h column, the norm's fold sums, the norm) reach the host through one pinned copy
    # and an event: the next iteration's M and A applies are queued before the host waits, so the host's
    # Givens step and the GPU's applies overlap (the last iteration's speculative apply is discarded)
    on_gpu = b.is_cuda
    hbuf = torch.empty(m + 5, dtype=torch.float64, pin_memory=on_gpu)
    ev = torch.cuda.Event() if on_gpu else None

    def head(j):
        """Z[j] = M V[j], w = A Z[j]."""
        Z[j] = Mop(V[j]) if Mop is not None else V[j]
        _apply_into(Aop, Z[j], w)

    while it < maxiter:
        beta = normr
        H = np.zeros((m + 1, m))
        cs, sn = np.zeros(m), np.zeros(m)
        g = np.zeros(m + 1)
        g[0] = beta
        torch.div(r, beta, out=V[0])
        vb[0:1] = bnd[0:1] / beta * _VB_SLACK   # (bnd[0] = max |r| from norm(r))
        k = 0
        head(0)
        for j in range(m):
            hs = None
            if fused and j + 1 <= 256:
                # CGS2 in three passes over the basis instead of four: h1 = V w; (w -= V^T h1, h2 = V w) in one pass;
                # w -= V^T h2
                K.amax(w, bnd[1:2])
                hs = K.dots(V, n, j + 1, w, vb, bnd[1:2]).clone()
                h = K.update_dots(V, n, j + 1, hs, w, vb, bnd[1:2])
                K.update(V, n, j + 1, h, w, w)
                hs = hs + h
            else:
                for _ in range(2):        # CGS2: h = V w, w -= V^T h, twice
                    K.amax(w, bnd[1:2])
                    h = K.dots(V, n, j + 1, w, vb, bnd[1:2])
                    K.update(V, n, j + 1, h, w, w)
                    hs = h.clone() if hs is None else hs + h
            K.amax(w, bnd[1:2])
            a = K.fold_sums(w, n, 1, w, bnd[1:2], bnd[1:2])
            hn_d = torch.sqrt((a[0:1] + a[1:2]) + a[2:3])    # _finish, then the norm, on the device
            # an exact breakdown (hn == 0) makes V[j+1] zero rather than NaN: the speculative head(j+1) below then runs M
            # and A on a finite vector (its result is discarded when the host sees hn == 0)
            inv = torch.where(hn_d > 0, torch.reciprocal(hn_d), torch.zeros_like(hn_d))
            torch.mul(w, inv, out=V[j + 1])
            vb[j + 1:j + 2] = bnd[1:2] * inv * _VB_SLACK      # |fl(w_i inv)| <= fl(max|w| inv): rounding is monotone
            hbuf[: j + 5].copy_(torch.cat([hs, a[:3], hn_d]), non_blocking=on_gpu)
            if on_gpu:
                ev.record()
            if j + 1 < m and it + 1 < maxiter:
                head(j + 1)           # speculative: queued behind the copy, runs while the host works
            if on_gpu:
                ev.synchronize()
            host = hbuf[: j + 5].tolist()
            hcol = np.asarray(host[: j + 1])
            hn = host[j + 4]
            H[: j + 1, j] = hcol
            H[j + 1, j] = hn
            for i in range(j):                          # apply previous Givens rotations
                t = cs[i] * H[i, j] + sn[i] * H[i + 1, j]
                H[i + 1, j] = -sn[i] * H[i, j] + cs[i] * H[i + 1, j]
                H[i, j] = t
            den = math.hypot(H[j, j], H[j + 1, j])
            cs[j], sn[j] = (1.0, 0.0) if den == 0.0 else (H[j, j] / den, H[j + 1, j] / den)
            H[j, j] = cs[j] * H[j, j] + sn[j] * H[j + 1, j]
            H[j + 1, j] = 0.0
            g[j + 1] = -sn[j] * g[j]
            g[j] = cs[j] * g[j]
            k = j + 1
            it += 1
            res = abs(g[j + 1])
            if residuals is not None:
                residuals.append(res)
            if callback is not None:
                callback(lincomb(x, Z, k, _solve_upper(H, g, k)))
            if res <= target or it >= maxiter or hn == 0.0:
                break
        x = lincomb(x, Z, k, _solve_upper(H, g, k))
        r = b - Aop(x)
        normr = norm(r, 0)
        if normr <= target:
            return x, 0
    return x, it


def _fgmres_dcgs2(Aop, Mop, b, x0, tol, m, maxiter, callback, residuals, K):
    """fgmres's restart cycles with DCGS2 orthogonalisation (see fgmres).  Iteration j of a cycle: w = A M u_j (queued
    speculatively in iteration j - 1), max |w|, ONE block product [V[0..j]] . [u_j, w] (fold sums, one sum-reduction), the
    scalars and both updates on the device (V[j] <- q_j, V[j+1] <- u_{j+1} / r_j), one pinned copy of s, z, r, c to the
    host, which completes H's column j - 1 (z / r + s, c / r + s_j, r') and its Givens rotation -- the residual
    estimate is one iteration behind the iteration that formed the column.  Z[j] = M u_j keeps the raw vector (norm
    ~ r_j): the Arnoldi relation A Z' = V H holds for Z'[j] = Z[j] / r_j, so the solution update scales y_j by 1 / r_j
    (w = A Z[j] is scaled by the same 1 / r_j inside the update: the raw vectors stay at the size of A M q_j)."""
    n = b.numel()
    f64 = dict(dtype=b.dtype, device=b.device)
    x = torch.zeros_like(b) if x0 is None else (
        x0.clone() if isinstance(x0, torch.Tensor) else torch.from_numpy(np.asarray(x0, dtype=np.float64)).to(b.device))
    bnd = torch.empty(2, **f64)            # [max |r| (norms), max |w|]

    def norm(v, slot):
        K.amax(v, bnd[slot:slot + 1])
        a = K.fold_sums(v, n, 1, v, bnd[slot:slot + 1], bnd[slot:slot + 1])
        return math.sqrt(_finish(a.cpu().tolist()))

    def lincomb(xv, Zm, k, y):
        ny = torch.from_numpy(-(np.asarray(y[:k], dtype=np.float64) * zsc[:k])).to(b.device)
        return K.update(Zm, n, k, ny, xv, torch.empty_like(xv))

    r = b - Aop(x)
    normr = norm(r, 0)
    if residuals is not None:
        residuals[:] = [normr]
    normb = norm(b, 1) or 1.0
    if normr < tol * normb:
        return x, 0
    target = tol * normr if normr != 0.0 else tol
    it = 0
    w = torch.empty_like(b)
    V = torch.empty(m + 1, n, **f64)
    Z = torch.empty(m, n, **f64)
    vb = torch.ones(m + 1, **f64)          # |q_i| <= 1; vb[j] = the raw u_j's a-priori bound while it is raw
    on_gpu = b.is_cuda
    hbuf = torch.empty(2 * m + 8, dtype=torch.float64, pin_memory=on_gpu)
    ev = torch.cuda.Event() if on_gpu else None

    def head(j):
        Z[j] = Mop(V[j]) if Mop is not None else V[j]
        _apply_into(Aop, Z[j], w)

    while it < maxiter:
        beta = normr
        H = np.zeros((m + 1, m))
        cs, sn = np.zeros(m), np.zeros(m)
        g = np.zeros(m + 1)
        g[0] = beta
        torch.div(r, beta, out=V[0])
        vb.fill_(1.0)
        zsc = np.ones(m)                        # Z'[i] = Z[i] * zsc[i] (1 / r_i)
        k = 0                                   # completed columns
        zc = None                               # column j - 1's first-pass part (z, c), completed in iteration j
        head(0)
        done = False
        cyc = [beta]                            # this cycle's residual estimates, from its initial residual
        for j in range(m + 1):
            form = j < m and it + (1 if j > 0 else 0) < maxiter   # column j will be formed (w = A M u_j is needed)
            ubound = vb[j:j + 1]
            if form:
                K.amax(w, bnd[1:2])
            else:
                bnd[1:2].zero_()                # (no w: its products are not used)
            acc = K.block_folds(V, n, j + 1, V[j], w, vb, ubound, bnd[1:2])
            hu, hw, P = K.dcgs2_update(V, n, j, acc, bnd[1:2], w, upd_w=form)
            vb[j:j + 1] = 1.0                   # V[j] is the unit vector q_j now
            if form:
                vb[j + 1:j + 2] = P[3:4]        # the raw u_{j+1}'s a-priori bound
            hbuf[: 2 * j + 6].copy_(torch.cat([hu, hw, P]), non_blocking=on_gpu)
            if on_gpu:
                ev.record()
            nxt = form and j + 1 < m and it + (1 if j > 0 else 0) + 1 < maxiter
            # head(j + 1) is speculative: queued behind the copy, it runs while the host completes column j - 1.  When
            # the estimates' rate says that column may be the last (the next estimate within 10x of the target), it
            # waits for the host instead: a converged solve then skips one apply (an mg:8 / mg:1 apply is ~8 ms at
            # 1024^2) for one host round trip (~0.25 ms) when it does not converge.  Only the timing changes, never
            # the values.
            late = nxt and len(cyc) >= 2 and cyc[-2] > 0.0 and cyc[-1] * (cyc[-1] / cyc[-2]) <= 10.0 * target
            if nxt and not late:
                head(j + 1)
            if on_gpu:
                ev.synchronize()
            host = hbuf[: 2 * j + 6].tolist()
            s_, z_ = host[:j], host[j + 1: 2 * j + 1]
            rj, rinvj, cj = host[2 * j + 2], host[2 * j + 3], host[2 * j + 4]
            # r_j = sqrt(hu_j - s.s) forced to 0 while the raw u_j is not zero: the difference cancelled because the
            # basis lost orthogonality (a stalling solve), not a happy breakdown -- the column's estimate |g| = 0 would
            # be false, so the iteration records the true residual of the restart the cycle ends with instead
            lost = j > 0 and rj == 0.0 and host[j] > 0.0
            if j < m:
                zsc[j] = rinvj
            if j > 0:                           # complete column j - 1: H = (z / r + s, c / r + s_{j-1}, r')
                zp, cp, ip = zc
                col = j - 1
                for i in range(col):
                    H[i, col] = zp[i] * ip + s_[i]
                H[col, col] = cp * ip + s_[col]
                H[j, col] = rj
                for i in range(col):            # previous Givens rotations
                    t = cs[i] * H[i, col] + sn[i] * H[i + 1, col]
                    H[i + 1, col] = -sn[i] * H[i, col] + cs[i] * H[i + 1, col]
                    H[i, col] = t
                den = math.hypot(H[col, col], H[col + 1, col])
                cs[col], sn[col] = (1.0, 0.0) if den == 0.0 else (H[col, col] / den, H[col + 1, col] / den)
                H[col, col] = cs[col] * H[col, col] + sn[col] * H[col + 1, col]
                H[col + 1, col] = 0.0
                g[col + 1] = -sn[col] * g[col]
                g[col] = cs[col] * g[col]
                k = j
                it += 1
                res = abs(g[col + 1])
                cyc.append(res)
                if residuals is not None and not lost:
                    residuals.append(res)
                if callback is not None:
                    callback(lincomb(x, Z, k, _solve_upper(H, g, k)))
                if res <= target or it >= maxiter or rj == 0.0:
                    done = True
                    break
            if not form:
                break
            if late:
                head(j + 1)                     # the deferred speculation: the cycle goes on
            zc = (z_, cj, rinvj)
        x = lincomb(x, Z, k, _solve_upper(H, g, k))
        r = b - Aop(x)
        normr = norm(r, 0)
        if lost and residuals is not None:
            residuals.append(normr)
        if normr <= target:
            return x, 0
        if not done and k == 0:
            break
    return x, it


def print_true_res_norm(A, b_vec):
    """Callback printing true residual norms (solve.py:161-170)."""
    iteration = 0
    op = _as_operator(A)
    nb = float(torch.linalg.vector_norm(b_vec))

    def callback(xk):
        nonlocal iteration
        iteration += 1
        res = float(torch.linalg.vector_norm(b_vec - op(xk)))
        print(f"GMRES Iteration {iteration}: True residual norm = {res}, Rel residual norm: {res / nb}")
    return callback


def solve_with_approx_schur_pc(n, xi, etan, etas, c, d, b_vec, u_vec, inner_F=None, inner_P=None,
                               tol=1e-8, maxiter=150, verbose=True):
    """solve.py:240-286: FGMRES on A with the approximate-commutator preconditioner.

    Returns (u_approx, info, residual history) with u_approx a host array.
    """
    from .utils import print_norms
    bp = MultiphaseBlockPreconditioner(n, xi, etan, etas)
    A, _, F, D, G = bp.get_big_A_matrix(c=c, d_u=d)
    pc = ApproxSchurPreconditioner(F, D, G, inner_F=inner_F, inner_P=inner_P)
    b = torch.from_numpy(np.ascontiguousarray(b_vec, dtype=np.float64)).to(pc.device)
    hist = []
    x, info = fgmres(A, b, M=pc, tol=tol, maxiter=maxiter,
                     callback=print_true_res_norm(A, b) if verbose else None, residuals=hist)
    u_approx = x.cpu().numpy()
    if verbose:
        print("\nPrinting error norms for solving Ax=b using fGMRES with approx schur complement as preconditioner:")
        print_norms(u_approx, u_vec, 1 / n, 1 / n, n)
    return u_approx, info, hist


def solve_without_pc(n, A, b_vec, u_vec, tol=1e-8, maxiter=100, verbose=True):
    """solve.py:202-208: FGMRES on A without a preconditioner (x0 = 0), then the error norms.

    A is the DeviceCSR from get_big_A_matrix; returns (u_approx, info, residual history)."""
    from .utils import print_norms
    b = torch.from_numpy(np.ascontiguousarray(b_vec, dtype=np.float64)).to(A.device)
    hist = []
    x, info = fgmres(A, b, x0=torch.zeros_like(b), M=None, tol=tol, maxiter=maxiter,
                     callback=print_true_res_norm(A, b) if verbose else None, residuals=hist)
    u_approx = x.cpu().numpy()
    if verbose:
        print("\nPrinting error norms for solving Ax=b using fGMRES without preconditioner:")
        print_norms(u_approx, u_vec, 1 / n, 1 / n, n)
    return u_approx, info, hist
