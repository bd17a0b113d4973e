"""Pin the CPU oracle against fixtures generated from the reference itself (tests/golden/).

Tolerances: matrix entries and vectors within 1e-12 relative infinity-norm (BASELINE.json
north_star); stencil patterns must cover every nonzero of the reference's dense matrices, and
entries the oracle keeps structurally where the reference holds an exact zero must be
negligible (<= 1e-12 of the matrix scale).
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_csr, golden_files, golden_params, load_golden, rel_inf

TOL = 1e-12

CASES = [os.path.basename(p) for p in golden_files()]


def _system(g, products=True):
    from oracle.stokes_oracle import StokesSystem
    return StokesSystem(**golden_params(g), products=products)


def assert_matrix_matches(ours, ref, tol=TOL):
    ours = sp.csr_matrix(ours)
    ref = sp.csr_matrix(ref)
    assert ours.shape == ref.shape
    ref_pat = set(zip(*ref.nonzero()))
    coo = ours.tocoo()
    our_pat = set(zip(coo.row.tolist(), coo.col.tolist()))
    assert ref_pat <= our_pat, f"missing {len(ref_pat - our_pat)} reference nonzeros"
    scale = max(abs(ref).max(), 1e-300)
    diff = abs(ours - ref).max()
    assert diff <= tol * scale, f"max |diff| {diff:.3e} > {tol:g} * {scale:.3e}"


@pytest.mark.parametrize("case", CASES)
def test_big_A_matrix(case, oracle_built):
    g = load_golden(os.path.join(os.path.dirname(__file__), "golden", case))
    big = "Ln_data" not in g
    sysm = _system(g, products=not big)
    assert_matrix_matches(sysm.A, golden_csr(g, "A"))
    if big:
        return
    assert_matrix_matches(sysm.F, golden_csr(g, "F"))
    assert_matrix_matches(sysm.D, golden_csr(g, "D"))
    assert_matrix_matches(sysm.G, golden_csr(g, "G"))
    for tag, is_ths in (("n", False), ("s", True)):
        L, D, XI, G = sysm.block_matrices(is_ths)
        assert_matrix_matches(L, golden_csr(g, "L" + tag))
        assert_matrix_matches(D, golden_csr(g, "D" + tag))
        assert_matrix_matches(XI, golden_csr(g, "XI" + tag))
        assert_matrix_matches(G, golden_csr(g, "G" + tag))


@pytest.mark.parametrize("case", [c for c in CASES if "n32" not in c])
def test_commutator_products(case, oracle_built):
    g = load_golden(os.path.join(os.path.dirname(__file__), "golden", case))
    sysm = _system(g)
    assert_matrix_matches(sysm.GtG, golden_csr(g, "GtG"))
    assert_matrix_matches(sysm.GtFG, golden_csr(g, "GtFG"))


@pytest.mark.parametrize("case", CASES)
def test_apply_matvec(case, oracle_built):
    """apply.py:72 b_approx = A @ u_vec on the manufactured solution."""
    from oracle import csr_oracle as co
    g = load_golden(os.path.join(os.path.dirname(__file__), "golden", case))
    sysm = _system(g, products=False)
    assert rel_inf(co.spmv(sysm.A, g["u_vec"]), g["Au"]) <= TOL


@pytest.mark.parametrize("case", [c for c in CASES if "n32" not in c])
def test_schur_apply_jacobi(case, oracle_built):
    from oracle.schur_oracle import Inner, approx_schur_apply
    g = load_golden(os.path.join(os.path.dirname(__file__), "golden", case))
    s = _system(g)
    for nf, npp in ((1, 1), (3, 2)):
        out = approx_schur_apply(s.F, s.D, s.G, s.GtG, s.GtFG, g["v"], Inner("jacobi", nf), Inner("jacobi", npp))
        assert rel_inf(out, g[f"schur_jacobi_{nf}_{npp}"]) <= 1e-11, (nf, npp)


@pytest.mark.parametrize("case", [c for c in CASES if "n32" not in c])
def test_inner_jacobi(case, oracle_built):
    from oracle.schur_oracle import Inner, diagonal, inner_solve
    g = load_golden(os.path.join(os.path.dirname(__file__), "golden", case))
    s = _system(g)
    nu = s.F.shape[0]
    xF = inner_solve(s.F, diagonal(s.F), Inner("jacobi", 4), g["v"][:nu])
    assert rel_inf(xF, g["jacobi_F_4"]) <= 1e-11
    xP = inner_solve(s.GtG, diagonal(s.GtG), Inner("jacobi", 4), g["v"][nu:])
    assert rel_inf(xP, g["jacobi_GtG_4"]) <= 1e-11


@pytest.mark.parametrize("case", [c for c in CASES if "n32" not in c and "n16" not in c])
def test_schur_apply_exact_inverses(case, oracle_built):
    """Composition of solve.py:257-277 with exact inner inverses (pseudo-inverse for the singular Gt_G)."""
    from oracle.schur_oracle import Inner, approx_schur_apply
    g = load_golden(os.path.join(os.path.dirname(__file__), "golden", case))
    s = _system(g)
    Fd = s.F.toarray()
    Pinv = np.linalg.pinv(s.GtG.toarray())
    out = approx_schur_apply(s.F, s.D, s.G, s.GtG, s.GtFG, g["v"], Inner("exact"), Inner("exact"),
                             F_inv=lambda r: np.linalg.solve(Fd, r), GtG_inv=lambda r: Pinv @ r)
    assert rel_inf(out, g["schur_exact"]) <= 1e-8


@pytest.mark.parametrize("case", [c for c in CASES if "n32" not in c])
def test_scipy_form_matches_oracle(case, oracle_built):
    """bench.py's scipy-form CPU baseline (scipy.sparse products) computes the oracle's apply, and the
    Jacobi case matches the reference's own composition fixture."""
    from oracle.schur_oracle import Inner, approx_schur_apply, approx_schur_apply_scipy, diagonal, gershgorin
    g = load_golden(os.path.join(os.path.dirname(__file__), "golden", case))
    s = _system(g)
    dF, dP = diagonal(s.F), diagonal(s.GtG)
    lf, lp = gershgorin(s.F, dF), gershgorin(s.GtG, dP)
    for iF, iP in ((Inner("jacobi", 3), Inner("jacobi", 2)),
                   (Inner("chebyshev", 4, lf / 30, lf), Inner("chebyshev", 4, lp / 30, lp))):
        ref = approx_schur_apply(s.F, s.D, s.G, s.GtG, s.GtFG, g["v"], iF, iP)
        out = approx_schur_apply_scipy(s.F, s.D, s.G, s.GtG, s.GtFG, g["v"], iF, iP, dF, dP)
        assert rel_inf(out, ref) <= 1e-12, iF.kind
    out = approx_schur_apply_scipy(s.F, s.D, s.G, s.GtG, s.GtFG, g["v"], Inner("jacobi", 3), Inner("jacobi", 2),
                                   dF, dP)
    assert rel_inf(out, g["schur_jacobi_3_2"]) <= 1e-11
