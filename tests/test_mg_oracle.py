"""CPU checks of the multigrid restatement (oracle/mg_oracle.py): transfer identities, Galerkin hierarchy,
V-cycle contraction, and the solve-level effect inside the approximate Schur preconditioner (solve.py:257-277,
with the multigrid the reference's comments point to at solve.py:266, 274)."""
import math

import numpy as np
import pytest


@pytest.fixture(scope="module")
def mo(oracle_built):
    from oracle import mg_oracle
    return mg_oracle


@pytest.mark.parametrize("n", [4, 6, 16])
def test_transfer_identities(mo, n):
    for fields in (mo.FIELDS_PRESSURE, mo.FIELDS_VELOCITY):
        P, R = mo.transfer(n, fields, "P"), mo.transfer(n, fields, "R")
        assert P.shape == (len(fields) * n * n, len(fields) * (n // 2) ** 2)
        assert np.array_equal(np.asarray(P.sum(axis=1)).ravel(), np.ones(P.shape[0]))   # interpolates constants
        assert (R != P.T).nnz == 0
        # 1D list lengths: cell 2, node 1 (even fine index) or 2 (odd); R the transposed lists (4 / 3)
        want = np.concatenate([np.outer([2, 2] * (n // 2) if ky == mo.CELL else [1, 2] * (n // 2),
                                        [2, 2] * (n // 2) if kx == mo.CELL else [1, 2] * (n // 2)).ravel()
                               for ky, kx in fields])
        assert np.array_equal(np.diff(P.indptr), want)
        assert P.nnz == np.count_nonzero(P.data)
        for M in (P, R):
            for r in range(M.shape[0]):
                cols = M.indices[M.indptr[r]:M.indptr[r + 1]]
                assert np.all(np.diff(cols) > 0)


def test_transfer_interpolates_linear_functions(mo):
    """Along a node axis P reproduces a linear function exactly away from the periodic seam; along a cell axis
    too (the weights are the linear interpolation weights at the fine positions)."""
    n = 16
    P = mo.p1d(n, mo.NODE)
    xc = 2.0 * np.arange(n // 2)
    xf = P @ xc
    assert np.allclose(xf[: n - 1], np.arange(n - 1))
    P = mo.p1d(n, mo.CELL)
    xc = 2.0 * np.arange(n // 2) + 1.0          # coarse cell centres in fine units (cell i at 2i + 1 - 1/2 ...)
    xf = P @ xc
    assert np.allclose(xf[1: n - 1], np.arange(1, n - 1) + 0.5)


def test_vcycle_contracts(mo):
    from oracle.stokes_oracle import StokesSystem
    S = StokesSystem(32, 1.0, 100.0, 1.0)
    rng = np.random.default_rng(0)
    for A, fields in ((S.F, mo.FIELDS_VELOCITY), (S.GtG, mo.FIELDS_PRESSURE)):
        M = mo.MgOracle(A, 32, fields)
        assert [m for _, m in M.ops] == [32, 16, 8]
        b = A @ rng.standard_normal(A.shape[0])
        x = np.zeros_like(b)
        for _ in range(4):
            x = x + M.solve(b - A @ x)
        rate = (np.linalg.norm(b - A @ x) / np.linalg.norm(b)) ** 0.25
        assert rate < 0.1, rate


def _fgmres_its(A, b, M, tol=1e-8, maxiter=150):
    """Right-preconditioned FGMRES iteration count (numpy; the host restatement used only by this test)."""
    n = b.size
    beta = np.linalg.norm(b)
    V = np.zeros((maxiter + 1, n))
    H = np.zeros((maxiter + 1, maxiter))
    V[0] = b / beta
    g = np.zeros(maxiter + 1)
    g[0] = beta
    cs, sn = np.zeros(maxiter), np.zeros(maxiter)
    for j in range(maxiter):
        w = A @ M(V[j])
        for _ in range(2):
            h = V[: j + 1] @ w
            w = w - V[: j + 1].T @ h
            H[: j + 1, j] += h
        H[j + 1, j] = np.linalg.norm(w)
        V[j + 1] = w / H[j + 1, j]
        for i in range(j):
            t = cs[i] * H[i, j] + sn[i] * H[i + 1, j]
            H[i + 1, j] = -sn[i] * H[i, j] + cs[i] * H[i + 1, j]
            H[i, j] = t
        den = math.hypot(H[j, j], H[j + 1, j])
        cs[j], sn[j] = H[j, j] / den, H[j + 1, j] / den
        H[j, j], H[j + 1, j] = den, 0.0
        g[j + 1], g[j] = -sn[j] * g[j], cs[j] * g[j]
        if abs(g[j + 1]) <= tol * beta:
            return j + 1
    return maxiter


def test_mg_preconditioner_beats_chebyshev(mo, oracle_built):
    """At 32^2 (eta_n = 100) the Schur preconditioner with one V-cycle per inner inverse needs far fewer FGMRES
    iterations than with 4 Chebyshev sweeps (the applies/s headline's inner solver)."""
    from oracle import csr_oracle as co
    from oracle.schur_oracle import Inner, approx_schur_apply, gershgorin
    from oracle.stokes_oracle import StokesSystem
    import mp_block_preconditioners_amd.utils as ut
    n = 32
    S = StokesSystem(n, 1.0, 100.0, 1.0)
    _, b = ut.manufactured_problem(n, etan=100.0, etas=1.0)
    dF, dP = S.F.diagonal(), S.GtG.diagonal()
    lF, lP = gershgorin(S.F, dF), gershgorin(S.GtG, dP)
    cheb = lambda v: approx_schur_apply(S.F, S.D, S.G, S.GtG, S.GtFG, v, Inner("chebyshev", 4, lF / 30, lF),
                                        Inner("chebyshev", 4, lP / 30, lP))
    oF = mo.MgOracle(S.F, n, mo.FIELDS_VELOCITY)
    oP = mo.MgOracle(S.GtG, n, mo.FIELDS_PRESSURE)
    nu = S.F.shape[0]

    def mg(v):
        Fv = oF.solve(v[:nu])
        xp = oP.solve(co.spmv(S.GtFG, oP.solve(co.spmv(S.D, Fv, v[nu:], mode=1))))
        return np.concatenate([oF.solve(co.spmv(S.G, xp), sub=Fv), xp])
    it_cheb, it_mg = _fgmres_its(S.A, b, cheb), _fgmres_its(S.A, b, mg)
    assert it_mg < 70 and it_mg < it_cheb, (it_mg, it_cheb)


@pytest.mark.parametrize("n", [32, 64])
def test_coarse_inverse_drops_the_pressure_null_space(mo, n):
    """mg.COARSE_RCOND: the coarsest Gt_G (periodic: constants in its null space) gets a rank m - 1 pseudo-inverse that
    maps constants to ~0; the coarsest F keeps full rank.  (At 1024^2 numpy's default cut kept Gt_G's roundoff-level
    constant mode and the pressure solve's output carried a ~1e17 constant: tools/coarse_spectrum.py.)"""
    from mp_block_preconditioners_amd import mg
    from oracle.stokes_oracle import StokesSystem
    assert mo.COARSE_RCOND == mg.COARSE_RCOND
    S = StokesSystem(n, 1.0, 100.0, 1.0, 1.0, -1.0, products=True)
    oP = mo.MgOracle(S.GtG, n, mo.FIELDS_PRESSURE, coarsest=8)
    oF = mo.MgOracle(S.F, n, mo.FIELDS_VELOCITY, coarsest=8)
    m = oP.coarse_inv.shape[0]
    assert np.linalg.matrix_rank(oP.coarse_inv, tol=1e-8 * np.abs(oP.coarse_inv).max()) == m - 1
    assert np.abs(oP.coarse_inv @ np.ones(m)).max() <= 1e-10 * np.abs(oP.coarse_inv).max()
    assert np.linalg.matrix_rank(oF.coarse_inv) == oF.coarse_inv.shape[0]
