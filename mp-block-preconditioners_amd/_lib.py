"""ctypes binding of libmpbp.so (include/mpbp.h).  Loading fails loudly: there is no CPU fallback."""
from __future__ import annotations

import ctypes
import os
from ctypes import (CFUNCTYPE, POINTER, Structure, byref, c_char_p, c_double, c_int, c_int32,
                    c_int64, c_void_p)

HERE = os.path.dirname(os.path.abspath(__file__))
# MPBP_LIB selects an experiment build of the same library (tools/build_variants.py); default: the product
LIB_PATH = os.environ.get("MPBP_LIB") or os.path.join(HERE, "lib", "libmpbp.so")

OP_A, OP_F, OP_D, OP_G = 0, 1, 2, 3
OP_L_N, OP_L_S, OP_D_N, OP_D_S, OP_G_N, OP_G_S, OP_XI_N, OP_XI_S = range(4, 12)
SPMV_STORE, SPMV_ADD, SPMV_RESID = 0, 1, 2
OK, ERR_ARG = 0, -1                    # mpbp.h return codes (MPBP_OK, MPBP_ERR_ARG)
SPMV_FAST = 0x100                     # mpbp_f_stencil_spmv: tolerance-mode F rows
NUMERICS_EXACT, NUMERICS_FAST = 0, 1  # mpbp_schur_plan.f_numerics
INNER_JACOBI, INNER_CHEBYSHEV, INNER_MG = 0, 1, 2
MG_CELL, MG_NODE = 0, 1
MG_P, MG_R = 0, 1
HALO_BEGIN, HALO_END = 0, 1
VEC_VELOCITY, VEC_PRESSURE = 0, 1
PG_D, PG_G, PG_GTG = 0, 1, 2
HALO_IN_ORDER, HALO_OVERLAP = 0, 1
BLOCK_ROWS, BLOCK_NNZ = 256, 4095


class MpbpError(RuntimeError):
    pass


class Csr(Structure):
    _fields_ = [("nrows", c_int32), ("ncols", c_int32), ("nnz", c_int64),
                ("row_ptr", c_void_p), ("col_idx", c_void_p), ("val", c_void_p)]


class RowBlocks(Structure):
    _fields_ = [("pairs", c_void_p), ("count", c_int32), ("reserved", c_int32), ("table", c_void_p)]


class Sell(Structure):
    _fields_ = [("nrows", c_int32), ("ncols", c_int32), ("nslices", c_int32), ("reserved", c_int32),
                ("slices", c_void_p), ("row_len", c_void_p), ("val", c_void_p), ("col", c_void_p)]


class RowPart(Structure):
    _fields_ = [("r0", c_int32), ("rows", c_int32), ("halo", c_int32), ("which", c_int32), ("ext", c_int32),
                ("oh", c_int32)]


class StokesParams(Structure):
    _fields_ = [("n", c_int32), ("xi", c_double), ("eta_n", c_double), ("eta_s", c_double),
                ("c", c_double), ("d_u", c_double), ("d_p", c_double), ("d_div", c_double)]


class InnerSolverC(Structure):
    _fields_ = [("kind", c_int32), ("sweeps", c_int32), ("lmin", c_double), ("lmax", c_double)]


class Svl(Structure):
    _fields_ = [("nfields", c_int32), ("m", c_int32), ("reach", c_int32), ("slots", c_int32),
                ("delta", c_void_p), ("vals", c_void_p), ("edge_rows", c_void_p), ("n_edge", c_int32),
                ("reserved", c_int32)]


class MgLevel(Structure):
    _fields_ = [("nrows", c_int32), ("pre", c_int32), ("post", c_int32), ("part_r0", c_int32),
                ("lmin", c_double), ("lmax", c_double), ("A", Csr), ("A_blocks", RowBlocks), ("diag", c_void_p),
                ("R", Csr), ("R_blocks", RowBlocks), ("P", Csr), ("P_blocks", RowBlocks),
                ("x", c_void_p), ("t", c_void_p), ("r", c_void_p), ("d", c_void_p), ("b", c_void_p),
                ("A_sell", Sell), ("R_sell", Sell), ("P_sell", Sell), ("halo_kind", c_int32), ("part_h", c_int32),
                ("A_svl", POINTER(Svl))]


HALO_FN = CFUNCTYPE(None, c_void_p, c_int32, c_void_p, c_int32, c_void_p)
HALO_PAIR_FN = CFUNCTYPE(None, c_void_p, c_void_p, c_void_p, c_void_p)
GATHER_FN = CFUNCTYPE(None, c_void_p, c_int32, c_void_p, c_void_p, c_void_p)


class KernelOpts(Structure):
    """mpbp_kernel_opts: which kernel form runs each step (include/mpbp.h "kernel choices")."""
    _fields_ = [("march_rows", c_int32), ("init_diag", c_int32), ("f_pair", c_int32), ("f_direct", c_int32),
                ("gtg_fused", c_int32), ("gtg_tpb", c_int32), ("gtg_drhs", c_int32), ("q13_sym", c_int32),
                ("f_tile", c_int32), ("f_solve", c_int32), ("mg_galerkin_mf", c_int32), ("mg_galerkin_mf_p", c_int32),
                ("pg_direct", c_int32), ("mg_group_rows", c_int32), ("mg_svl", c_int32), ("mg_mf_transfer", c_int32),
                ("csr_table", c_int32), ("mg_fuse_l0", c_int32), ("mg_coarse_tree", c_int32),
                ("f_solve_tile", c_int32), ("q13_mf", c_int32), ("mg_fuse_small", c_int32),
                ("gtg_solve_tile", c_int32), ("reserved", c_int32 * 1)]


def kernel_opts(overrides=None) -> KernelOpts:
    """A plan's kernel choices: this thread's current ones (a kernel_options block, else the process defaults set by
    mpbp_set_*) at this moment, with `overrides` (a dict of KernelOpts field names) applied.  Unknown names raise."""
    o = KernelOpts()
    lib().mpbp_kernel_opts_default(ctypes.byref(o))
    names = {f for f, _ in KernelOpts._fields_ if f != "reserved"}
    for k, v in (overrides or {}).items():
        if k not in names:
            raise ValueError(f"unknown kernel option {k!r} (known: {sorted(names)})")
        setattr(o, k, int(v))
    return o


# every KernelOpts a kernel_options block has installed and not yet restored: the C thread-local pointer refers to the
# struct, so it must outlive the block even when __exit__ never runs (an abandoned generator, a by-hand __enter__)
_INSTALLED: list = []


class kernel_options:
    """Context manager: kernel choices for this thread inside the block -- the current ones with `overrides` applied
    (mpbp_kernel_opts_set_thread): the plan-less entry points (mpbp_spmv, mpbp_f_stencil_*, mpbp_pg_stencil_*, ...)
    use them, and plans created inside the block start from them; the previous thread choice is restored on exit.
    Plans created before keep their own copies."""

    def __init__(self, **overrides):
        self.opts = kernel_opts(overrides)
        self._prev = ctypes.c_void_p()
        self._active = False

    def __enter__(self):
        if self._active:   # a second entry would overwrite _prev: the earlier choice could never be restored
            raise RuntimeError("kernel_options: this block is already active (use a new instance to nest)")
        check(lib().mpbp_kernel_opts_set_thread(ctypes.byref(self.opts), ctypes.byref(self._prev)))
        self._active = True
        _INSTALLED.append(self.opts)
        return self.opts

    def __exit__(self, *exc):
        check(lib().mpbp_kernel_opts_set_thread(self._prev, None))
        self._active = False
        for i, o in enumerate(_INSTALLED):
            if o is self.opts:
                del _INSTALLED[i]
                break
        return False


class Mg(Structure):
    _fields_ = [("nlevels", c_int32), ("cycles", c_int32), ("levels", POINTER(MgLevel)), ("coarse_inv", Csr),
                ("coarse_inv_blocks", RowBlocks), ("coarse_dense", c_void_p),
                ("part_levels", c_int32), ("gather_kind", c_int32), ("halo", HALO_FN), ("halo_ctx", c_void_p),
                ("gather", GATHER_FN), ("tr_nfields", c_int32), ("tr_n0", c_int32), ("tr_ky", c_int32 * 8),
                ("tr_kx", c_int32 * 8), ("opts", POINTER(KernelOpts))]


class SchurPlan(Structure):
    _fields_ = [("nu", c_int32), ("np", c_int32), ("nu_ext", c_int32), ("np_ext", c_int32),
                ("F", Csr), ("D", Csr), ("G", Csr), ("GtG", Csr), ("GtFG", Csr),
                ("F_int", RowBlocks), ("F_bnd", RowBlocks), ("D_int", RowBlocks), ("D_bnd", RowBlocks),
                ("G_int", RowBlocks), ("G_bnd", RowBlocks), ("P_int", RowBlocks), ("P_bnd", RowBlocks),
                ("Q_int", RowBlocks), ("Q_bnd", RowBlocks),
                ("diag_F", c_void_p), ("diag_P", c_void_p),
                ("inner_F", InnerSolverC), ("inner_P", InnerSolverC),
                ("wu", c_void_p * 4), ("wu_owned", c_void_p), ("wp", c_void_p * 7),
                ("halo", HALO_FN), ("halo_ctx", c_void_p),
                ("prof_events", c_void_p), ("prof_capacity", c_int32), ("prof_count", POINTER(c_int32)),
                ("use_sell", c_int32),
                ("Fs_int", Sell), ("Fs_bnd", Sell), ("Ds_int", Sell), ("Ds_bnd", Sell), ("Gs_int", Sell),
                ("Gs_bnd", Sell), ("Ps_int", Sell), ("Ps_bnd", Sell), ("Qs_int", Sell), ("Qs_bnd", Sell),
                ("f_stencil", c_int32), ("f_prm", StokesParams), ("f_cell", c_void_p), ("f_uface", c_void_p),
                ("f_vface", c_void_p), ("f_part", RowPart), ("pg_stencil", c_int32), ("p_part", RowPart),
                ("halo_first", c_int32), ("ca", c_int32), ("ca_reach_q", c_int32), ("wu_ext", c_void_p),
                ("diag_F_ext", c_void_p), ("diag_P_ext", c_void_p), ("halo_pair", HALO_PAIR_FN),
                ("q13", c_void_p), ("q13_n", c_int32), ("mg_F", POINTER(Mg)), ("mg_P", POINTER(Mg)),
                ("fuse_g", c_int32), ("f_numerics", c_int32), ("opts", POINTER(KernelOpts))]


_P = c_void_p
_SIGNATURES = {
    "mpbp_version": ([], c_char_p),
    "mpbp_last_error": ([], c_char_p),
    "mpbp_stokes_theta": ([c_int32, _P, _P, _P, _P], c_int),
    "mpbp_stokes_rows": ([c_int32, c_int32], c_int64),
    "mpbp_stokes_cols": ([c_int32, c_int32], c_int64),
    "mpbp_stokes_count": ([POINTER(StokesParams), c_int32, _P, _P, _P], c_int),
    "mpbp_stokes_fill": ([POINTER(StokesParams), c_int32, _P, _P, _P, _P, _P, _P, _P], c_int),
    "mpbp_exclusive_scan": ([_P, _P, c_int64, POINTER(c_int64), _P], c_int),
    "mpbp_spgemm_count": ([POINTER(Csr), POINTER(Csr), _P, _P], c_int),
    "mpbp_spgemm_fill": ([POINTER(Csr), POINTER(Csr), c_double, _P, _P, _P, _P], c_int),
    "mpbp_plan_row_blocks": ([_P, c_int32, c_int32, _P, c_int64], c_int64),
    "mpbp_csr_diag": ([POINTER(Csr), c_int32, _P, POINTER(c_int32), _P], c_int),
    "mpbp_gershgorin": ([POINTER(Csr), _P, POINTER(c_double), _P], c_int),
    "mpbp_csr_extract_count": ([POINTER(Csr), _P, c_int32, _P, _P], c_int),
    "mpbp_csr_extract_fill": ([POINTER(Csr), _P, c_int32, _P, _P, _P, _P, _P], c_int),
    "mpbp_spmv": ([POINTER(Csr), POINTER(RowBlocks), c_int32, _P, _P, _P, _P], c_int),
    "mpbp_spmv_seg": ([POINTER(Csr), POINTER(RowBlocks), c_int32, _P, _P, _P, _P], c_int),
    "mpbp_jacobi_init": ([c_int32, _P, _P, _P, _P, _P], c_int),
    "mpbp_jacobi_step": ([POINTER(Csr), POINTER(RowBlocks), _P, _P, _P, _P, _P, _P], c_int),
    "mpbp_cheb_init": ([c_int32, _P, _P, c_double, _P, _P, _P, _P], c_int),
    "mpbp_cheb_step": ([POINTER(Csr), POINTER(RowBlocks), _P, _P, _P, c_double, c_double, _P, _P, _P, _P],
                       c_int),
    "mpbp_cheb_coeffs": ([c_double, c_double, c_int32, _P, _P], c_int),
    "mpbp_schur_apply": ([POINTER(SchurPlan), _P, _P, _P], c_int),
    "mpbp_sell_plan": ([_P, _P, c_int32, _P, c_int64, POINTER(c_int64)], c_int64),
    "mpbp_sell_fill": ([POINTER(Csr), _P, c_int32, _P, _P, _P, _P], c_int),
    "mpbp_sell_spmv": ([POINTER(Sell), c_int32, _P, _P, _P, _P], c_int),
    "mpbp_sell_jacobi_step": ([POINTER(Sell), _P, _P, _P, _P, _P, _P], c_int),
    "mpbp_sell_cheb_step": ([POINTER(Sell), _P, _P, _P, c_double, c_double, _P, _P, _P, _P], c_int),
    "mpbp_f_stencil_spmv": ([POINTER(StokesParams), _P, _P, _P, POINTER(RowPart), c_int32, _P, _P, _P, _P], c_int),
    "mpbp_f_stencil_jacobi_step": ([POINTER(StokesParams), _P, _P, _P, POINTER(RowPart), _P, _P, _P, _P, _P],
                                   c_int),
    "mpbp_f_stencil_cheb_step": ([POINTER(StokesParams), _P, _P, _P, POINTER(RowPart), _P, _P, c_double, c_double,
                                  _P, _P, _P, _P], c_int),
    "mpbp_pg_stencil_spmv": ([POINTER(StokesParams), _P, POINTER(RowPart), c_int32, c_int32, _P, _P, _P, _P], c_int),
    "mpbp_gtg_stencil_jacobi_step": ([POINTER(StokesParams), _P, POINTER(RowPart), _P, _P, _P, _P, _P], c_int),
    "mpbp_gtg_stencil_cheb_step": ([POINTER(StokesParams), _P, POINTER(RowPart), _P, _P, c_double, c_double, _P, _P,
                                    _P, _P], c_int),
    "mpbp_rccl_unique_id": ([ctypes.c_char_p, _P], c_int),
    "mpbp_halo_create": ([ctypes.c_char_p, _P, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                          POINTER(c_void_p)], c_int),
    "mpbp_halo_create_shared": ([_P, c_int32, c_int32, c_int32, c_int32, c_int32, POINTER(c_void_p)], c_int),
    "mpbp_halo_comm": ([_P], c_void_p),
    "mpbp_halo_comm_refs": ([_P], c_int),
    "mpbp_halo_destroy": ([_P], None),
    "mpbp_halo_exchange": ([_P, c_int32, _P, c_int32, _P], None),
    "mpbp_halo_exchange_pair": ([_P, _P, _P, _P], None),
    "mpbp_halo_status": ([_P], c_int),
    "mpbp_halo_set_mode": ([_P, c_int32], c_int),
    "mpbp_halo_last_error": ([_P], c_char_p),
    "mpbp_halo_add_kind": ([_P, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32], c_int),
    "mpbp_halo_add_gather": ([_P, c_int32, c_int32, _P, _P], c_int),
    "mpbp_halo_allgather": ([_P, c_int32, _P, _P, _P], None),
    "mpbp_kernel_opts_default": ([POINTER(KernelOpts)], None),
    "mpbp_mg_level1_apply": ([POINTER(SchurPlan), c_int32, c_int32, _P, _P, _P, _P], c_int),
    "mpbp_rdot2": ([_P, c_int64, c_int32, _P, _P, c_int64, c_int64, _P, _P, _P, _P, _P, _P], c_int),
    "mpbp_dcgs2_update": ([_P, c_int64, c_int32, _P, _P, _P, c_int64, c_int32, _P, _P, _P, _P], c_int),
    "mpbp_hbm_stream": ([_P, c_int64, c_int32, _P, _P], c_int),
    "mpbp_gtg_stencil_cheb_solve": ([POINTER(StokesParams), _P, _P, _P, c_double, c_double, c_int32, _P, _P], c_int),
    "mpbp_kernel_opts_set_thread": ([c_void_p, c_void_p], c_int),
    "mpbp_q13_asymmetry": ([c_int32, _P, POINTER(c_double), _P], c_int),
    "mpbp_set_march_rows": ([c_int32], c_int),
    "mpbp_set_init_diag": ([c_int32], c_int),
    "mpbp_set_f_pair": ([c_int32], c_int),
    "mpbp_set_f_direct": ([c_int32], c_int),
    "mpbp_set_gtg_fused": ([c_int32], c_int),
    "mpbp_set_f_tile": ([c_int32], c_int),
    "mpbp_set_f_solve": ([c_int32], c_int),
    "mpbp_set_gtg_drhs": ([c_int32], c_int),
    "mpbp_set_q13_sym": ([c_int32], c_int),
    "mpbp_set_mg_galerkin_mf_p": ([c_int32], c_int),
    "mpbp_stokes_count_rows": ([POINTER(StokesParams), c_int32, _P, _P, c_int32, _P, _P], c_int),
    "mpbp_stokes_fill_rows": ([POINTER(StokesParams), c_int32, _P, _P, _P, _P, c_int32, _P, _P, _P, _P], c_int),
    "mpbp_set_mg_galerkin_mf": ([c_int32], c_int),
    "mpbp_set_pg_direct": ([c_int32], c_int),
    "mpbp_set_mg_group_rows": ([c_int32], c_int),
    "mpbp_set_mg_svl": ([c_int32], c_int),
    "mpbp_set_mg_mf_transfer": ([c_int32], c_int),
    "mpbp_set_csr_table": ([c_int32], c_int),
    "mpbp_q13_build": ([POINTER(Csr), c_int32, c_void_p, c_void_p], c_int),
    "mpbp_q13_build_rows": ([POINTER(Csr), c_int32, c_int32, c_void_p, c_void_p], c_int),
    "mpbp_svl_spmv": ([POINTER(Svl), POINTER(Csr), c_int32, _P, _P, _P, _P], c_int),
    "mpbp_svl_cheb_step": ([POINTER(Svl), POINTER(Csr), _P, _P, _P, c_double, c_double, _P, _P, _P, _P], c_int),
    "mpbp_q13_spmv": ([c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "mpbp_mg_transfer_count": ([c_int32, c_int32, _P, c_int32, _P, _P], c_int),
    "mpbp_mg_transfer_fill": ([c_int32, c_int32, _P, c_int32, _P, _P, _P, _P], c_int),
    "mpbp_mg_transfer_rows_count": ([c_int32, c_int32, _P, c_int32, _P, c_int32, _P, _P], c_int),
    "mpbp_mg_transfer_rows_fill": ([c_int32, c_int32, _P, c_int32, _P, c_int32, _P, _P, _P, _P], c_int),
    "mpbp_mg_solve": ([POINTER(Mg), _P, _P, _P, _P], c_int),
    "mpbp_gather": ([c_int32, _P, _P, _P, _P], c_int),
    "mpbp_scatter": ([c_int32, _P, _P, _P, _P], c_int),
    "mpbp_event_create": ([POINTER(c_void_p)], c_int),
    "mpbp_event_create_scoped": ([POINTER(c_void_p), c_int32], c_int),
    "mpbp_event_record": ([c_void_p, c_void_p], c_int),
    "mpbp_event_destroy": ([_P], c_int),
    "mpbp_event_elapsed_ms": ([_P, _P, POINTER(ctypes.c_float)], c_int),
    "mpbp_gs_dot": ([_P, c_int64, c_int32, _P, c_int64, _P, _P, _P], c_int),
    "mpbp_gs_part_size": ([c_int64, c_int32], c_int64),
    "mpbp_gs_update": ([_P, c_int64, c_int32, _P, _P, c_int64, _P, _P], c_int),
    "mpbp_rdot": ([_P, c_int64, c_int32, _P, c_int64, c_int64, _P, _P, _P, _P, _P], c_int),
    "mpbp_rdot_part_size": ([c_int64, c_int32], c_int64),
    "mpbp_gs_update_rdot": ([_P, c_int64, c_int32, _P, _P, c_int64, c_int64, _P, _P, _P, _P, _P, _P], c_int),
    "mpbp_rdot_finish": ([c_int32, _P, _P, _P], c_int),
    "mpbp_absmax": ([_P, c_int64, _P, _P], c_int),
}

_lib = None


def lib():
    """The loaded libmpbp.so; raises MpbpError if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MpbpError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                            f"g.build()'` (hipcc --offload-arch=gfx950).  There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGNATURES.items():
            # a library built from older sources lacks the newest entry points: calling one raises (AttributeError),
            # everything else stays usable; tests/test_abi.py checks that the built library exports every symbol
            fn = getattr(L, name, None)
            if fn is None:
                continue
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def check(rc):
    if rc < 0:
        raise MpbpError(f"libmpbp error {rc}: {lib().mpbp_last_error().decode()}")
    return rc


def exported_symbols():
    return list(_SIGNATURES)


def ptr(t):
    """Device (or host) address of a torch tensor / numpy array, or None."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        return ctypes.c_void_p(t.data_ptr())
    return t.ctypes.data_as(ctypes.c_void_p)


def stream_handle(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


__all__ = ["lib", "check", "ptr", "stream_handle", "MpbpError", "Csr", "RowBlocks", "Sell", "RowPart", "StokesParams",
           "InnerSolverC", "SchurPlan", "KernelOpts", "kernel_opts", "kernel_options", "HALO_FN", "GATHER_FN", "byref",
           "Mg", "MgLevel"]
