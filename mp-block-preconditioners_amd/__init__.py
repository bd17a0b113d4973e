"""mp-block-preconditioners on MI355X: the multiphase-Stokes operator and its approximate-commutator
block preconditioner, applied by hand-written HIP kernels for gfx950 (libmpbp.so, C ABI in
include/mpbp.h).  Import name: ``mp_block_preconditioners_amd`` (a symlink to this directory).
"""
from ._lib import MpbpError, lib
from .csr import DeviceCSR, DeviceSELL, spgemm
from .mg import FIELDS_PRESSURE, FIELDS_VELOCITY, Multigrid
from .preconditioner import MultiphaseBlockPreconditioner, thn, ths
from .solve import (ApproxSchurPreconditioner, InnerSolver, fgmres, print_true_res_norm,
                    solve_with_approx_schur_pc, solve_without_pc)
from .utils import (fill_sol_and_RHS_vecs, manufactured_problem, manufactured_problem_constant, max_norm, print_norms, weighted_L1,
                    weighted_L2)

__all__ = [
    "MpbpError", "lib", "DeviceCSR", "DeviceSELL", "spgemm", "MultiphaseBlockPreconditioner", "thn", "ths",
    "ApproxSchurPreconditioner", "InnerSolver", "fgmres", "print_true_res_norm",
    "solve_with_approx_schur_pc", "solve_without_pc", "fill_sol_and_RHS_vecs", "manufactured_problem", "manufactured_problem_constant", "max_norm",
    "print_norms", "weighted_L1", "weighted_L2", "Multigrid", "FIELDS_VELOCITY", "FIELDS_PRESSURE",
]
