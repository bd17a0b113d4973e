"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the reference fixtures.

Bars (BASELINE.json north_star):
* CSR indexing (row_ptr, col_idx) bit-exact against the oracle;
* values bit-exact against the oracle when both are fed the same thn tables (same IEEE operations,
  same order, no FMA), and within 1e-12 relative infinity-norm of the reference's fp64 results;
* at the BASELINE sizes (1024^2), where the oracle is too slow to run whole, size-independent
  properties: linearity and determinism of the apply, the O(h^2) consistency of A on the
  manufactured solution (the full 1024^2 assembly against the oracle: test_gpu_configs.py).
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_csr, golden_files, golden_params, golden_tables, load_golden, rel_inf

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(oracle_built):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _mp():
    import mp_block_preconditioners_amd as mp
    return mp


def _oracle_system(n, tables=None, **kw):
    from oracle.stokes_oracle import StokesSystem
    return StokesSystem(n, tables=tables, **kw)


def _same_csr(dev, ref):
    got = dev.to_scipy()
    ref = sp.csr_matrix(ref)
    assert got.shape == ref.shape
    assert np.array_equal(got.indptr, ref.indptr), "row_ptr differs"
    assert np.array_equal(got.indices, ref.indices), "col_idx differs"
    assert np.array_equal(got.data.view(np.uint64), ref.data.view(np.uint64)), \
        f"values differ (max {np.max(np.abs(got.data - ref.data)):.3e})"


def _cuda(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()


def _bits_equal(a, b):
    a = a.cpu().numpy() if hasattr(a, "cpu") else np.asarray(a)
    return np.array_equal(np.asarray(a, dtype=np.float64).view(np.uint64), np.asarray(b, dtype=np.float64).view(np.uint64))


PARAMS = dict(xi=1.0, eta_n=100.0, eta_s=1.0, c=1.0, d_u=-1.0, d_p=1.0, d_div=-1.0)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 16, 64])
def test_theta_tables_match_oracle(n):
    from oracle.stokes_oracle import theta_tables
    bp = _mp().MultiphaseBlockPreconditioner(n, 1.0, 1.0, 1.0)
    for got, ref in zip(bp.theta_tables(), theta_tables(n)):
        assert rel_inf(got.cpu().numpy(), ref) <= 4e-16


@pytest.mark.parametrize("n", [1, 2, 3, 4, 8, 33, 128])
def test_assembly_bit_exact(n):
    mp = _mp()
    from oracle.stokes_oracle import theta_tables
    tabs = theta_tables(n)
    osys = _oracle_system(n, tables=tabs, products=False, **PARAMS)
    bp = mp.MultiphaseBlockPreconditioner(n, PARAMS["xi"], PARAMS["eta_n"], PARAMS["eta_s"])
    bp.set_theta_tables(*tabs)
    A, S, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    assert S is None
    _same_csr(A, osys.A)
    _same_csr(F, osys.F)
    _same_csr(D, osys.D)
    _same_csr(G, osys.G)
    for is_ths in (False, True):
        for dev, ref in zip(bp.get_block_matrices(is_ths), osys.block_matrices(is_ths)):
            _same_csr(dev, ref)


@pytest.mark.parametrize("path", golden_files(), ids=os.path.basename)
def test_assembly_against_reference(path):
    """GPU-computed thn tables + GPU assembly vs the reference's dense matrices (1e-12)."""
    mp = _mp()
    from test_oracle_golden import assert_matrix_matches
    g = load_golden(path)
    p = golden_params(g)
    bp = mp.MultiphaseBlockPreconditioner(p["n"], p["xi"], p["eta_n"], p["eta_s"])
    if golden_tables(g) is not None:
        bp.set_theta_tables(*golden_tables(g))
    A, _, F, D, G = bp.get_big_A_matrix(c=p["c"], d_u=p["d_u"])
    assert_matrix_matches(A.to_scipy(), golden_csr(g, "A"))
    assert rel_inf(A.matvec(_cuda(g["u_vec"])).cpu().numpy(), g["Au"]) <= 1e-12     # apply.py:72
    if "F_data" in g:
        assert_matrix_matches(F.to_scipy(), golden_csr(g, "F"))
        GtG, GtFG = bp.commutator_products(F, D, G)
        assert_matrix_matches(GtG.to_scipy(), golden_csr(g, "GtG"))
        assert_matrix_matches(GtFG.to_scipy(), golden_csr(g, "GtFG"))


@pytest.mark.parametrize("n", [3, 16, 48])
def test_spgemm_bit_exact(n):
    mp = _mp()
    from oracle import csr_oracle as co
    osys = _oracle_system(n, **PARAMS)
    F, D, G = (mp.DeviceCSR.from_scipy(M) for M in (osys.F, osys.D, osys.G))
    GtG, GtFG = mp.MultiphaseBlockPreconditioner.commutator_products(F, D, G)
    _same_csr(GtG, osys.GtG)
    _same_csr(GtFG, osys.GtFG)
    _same_csr(mp.spgemm(F, G, alpha=2.5), co.spgemm(osys.F, osys.G, alpha=2.5))


@pytest.mark.parametrize("n", [2, 16, 100])
def test_spmv_bit_exact(n):
    mp = _mp()
    from oracle import csr_oracle as co
    osys = _oracle_system(n, products=False, **PARAMS)
    rng = np.random.default_rng(n)
    for M in (osys.A, osys.F, osys.D, osys.G):
        dM = mp.DeviceCSR.from_scipy(M)
        x = rng.standard_normal(M.shape[1])
        z = rng.standard_normal(M.shape[0])
        dS = dM.to_sell()
        for mode in (0, 1, 2):
            ref = co.spmv(M, x, z, mode=mode)
            y = dM.matvec(_cuda(x), mode=mode, z=_cuda(z))
            assert _bits_equal(y, ref), (M.shape, mode)
            y = dS.matvec(_cuda(x), mode=mode, z=_cuda(z))
            assert _bits_equal(y, ref), ("sell", M.shape, mode)
        h1 = dM @ x                                   # host vector in / out (page-locked staging)
        h2 = dM @ (2.0 * x)
        assert np.array_equal(h1, co.spmv(M, x)) and np.array_equal(h2, co.spmv(M, 2.0 * x))


@pytest.mark.parametrize("maxlen", [40, 255])
def test_sell_ragged_rows_and_partial_slices(maxlen):
    """SELL-64 with ragged rows (0..maxlen entries: past the first 16-entry batch, up to the layout's 255),
    partial slices, row ranges, a slice of uniform long rows (multigrid coarse operators), every epilogue."""
    mp = _mp()
    from oracle import csr_oracle as co
    rng = np.random.default_rng(11 + maxlen)
    lengths = rng.integers(0, maxlen + 1, size=1000)
    lengths[:64] = 0
    lengths[128:192] = maxlen
    rows = np.repeat(np.arange(lengths.size), lengths)
    M = sp.csr_matrix((rng.standard_normal(rows.size), (rows, rng.integers(0, 3000, size=rows.size))),
                      shape=(lengths.size, 3000))
    M.sum_duplicates()
    x = rng.standard_normal(3000)
    dM = mp.DeviceCSR.from_scipy(M)
    ref = co.spmv(M, x)
    assert _bits_equal(dM.to_sell().matvec(_cuda(x)), ref)
    y = torch.full((M.shape[0],), 7.0, dtype=torch.float64, device="cuda")
    dM.to_sell([(3, 100), (500, 1000)]).matvec(_cuda(x), out=y)
    got = y.cpu().numpy()
    sel = np.r_[3:100, 500:1000]
    assert _bits_equal(got[sel], ref[sel]) and np.all(got[np.r_[0:3, 100:500]] == 7.0)
    z = rng.standard_normal(M.shape[0])
    for mode in (1, 2):
        assert _bits_equal(dM.to_sell().matvec(_cuda(x), mode=mode, z=_cuda(z)), co.spmv(M, x, z, mode=mode)), mode


def test_spmv_long_rows_and_empty_rows():
    """Rows longer than a row block's LDS stage (single-row blocks) and empty rows: the per-wave kernel sums a
    long row chunk after chunk in order (bit-exact)."""
    mp = _mp()
    from oracle import csr_oracle as co
    rng = np.random.default_rng(7)
    lengths = rng.integers(0, 30, size=2000)
    lengths[[5, 777, 1999]] = [9000, 4096, 20000]
    lengths[[0, 10, 11]] = 0
    rows = np.repeat(np.arange(lengths.size), lengths)
    cols = rng.integers(0, 50000, size=rows.size)
    M = sp.csr_matrix((rng.standard_normal(rows.size), (rows, cols)), shape=(lengths.size, 50000))
    M.sum_duplicates()
    x = rng.standard_normal(50000)
    y = mp.DeviceCSR.from_scipy(M).matvec(_cuda(x)).cpu().numpy()
    ref = M @ x
    assert rel_inf(y, ref) <= 1e-13
    assert y[0] == 0.0 and y[10] == 0.0
    assert _bits_equal(y, co.spmv(M, x))


@pytest.mark.parametrize("maxlen", [13, 40, 200])
def test_csr_wave_chunks_ragged_bit_exact(maxlen):
    """Ragged rows whose 64-row wave ranges exceed one 768-entry chunk (rows straddle chunk edges,
    odd starts), partial last wave, empty rows, all three epilogue modes; bit-exact vs the oracle."""
    mp = _mp()
    from oracle import csr_oracle as co
    rng = np.random.default_rng(maxlen)
    lengths = rng.integers(0, maxlen + 1, size=3001)
    lengths[:70] = 0
    lengths[100:164] = maxlen
    rows = np.repeat(np.arange(lengths.size), lengths)
    M = sp.csr_matrix((rng.standard_normal(rows.size), (rows, rng.integers(0, 4000, size=rows.size))),
                      shape=(lengths.size, 4000))
    M.sum_duplicates()
    x, z = rng.standard_normal(4000), rng.standard_normal(lengths.size)
    dM = mp.DeviceCSR.from_scipy(M)
    for mode in (0, 1, 2):
        assert _bits_equal(dM.matvec(_cuda(x), mode=mode, z=_cuda(z)), co.spmv(M, x, z, mode=mode)), mode


@pytest.mark.parametrize("n", [4, 32])
def test_inner_steps_bit_exact(n):
    mp = _mp()
    from mp_block_preconditioners_amd import _lib
    from mp_block_preconditioners_amd._lib import check, lib, ptr, stream_handle
    from oracle import csr_oracle as co
    import ctypes
    osys = _oracle_system(n, **PARAMS)
    rng = np.random.default_rng(3)
    for M in (osys.F, osys.GtG):
        dM = mp.DeviceCSR.from_scipy(M)
        diag = M.diagonal().copy()
        b, x, d0, sub = (rng.standard_normal(M.shape[0]) for _ in range(4))
        tb, tx, tdiag, tsub = _cuda(b), _cuda(x), _cuda(diag), _cuda(sub)
        out = torch.empty_like(tb)
        blk = dM.blocks.cstruct()
        check(lib().mpbp_jacobi_step(ctypes.byref(dM.cstruct()), ctypes.byref(blk), ptr(tx), ptr(tb), ptr(tdiag),
                                     ptr(tsub), ptr(out), stream_handle()))
        assert _bits_equal(out, co.jacobi_step(M, x, b, diag, sub))
        td = _cuda(d0)
        d_ref = d0.copy()
        check(lib().mpbp_cheb_step(ctypes.byref(dM.cstruct()), ctypes.byref(blk), ptr(tx), ptr(tb), ptr(tdiag),
                                   0.3, 1.7, ptr(td), None, ptr(out), stream_handle()))
        ref = co.cheb_step(M, x, b, diag, 0.3, 1.7, d_ref)
        assert _bits_equal(out, ref) and _bits_equal(td, d_ref)


INNERS = [("jacobi", 1, "jacobi", 1), ("jacobi", 3, "jacobi", 2), ("chebyshev", 4, "chebyshev", 4),
          ("chebyshev", 6, "jacobi", 3)]


@pytest.mark.parametrize("layout", ["sell", "csr"])
@pytest.mark.parametrize("n", [3, 16, 64])
@pytest.mark.parametrize("inner", INNERS, ids=lambda t: f"{t[0]}{t[1]}-{t[2]}{t[3]}")
def test_schur_apply_bit_exact(n, inner, layout):
    """mpbp_schur_apply vs the oracle's restatement of approx_schur_op (solve.py:257-277)."""
    mp = _mp()
    from oracle.schur_oracle import Inner, approx_schur_apply, diagonal, gershgorin
    osys = _oracle_system(n, **PARAMS)
    kf, sf, kp, spp = inner
    pc = mp.ApproxSchurPreconditioner(osys.F, osys.D, osys.G, osys.GtG, osys.GtFG,
                                      inner_F=mp.InnerSolver(kf, sf), inner_P=mp.InnerSolver(kp, spp),
                                      layout=layout)
    # the oracle uses the bounds the GPU computed (Gershgorin on the GPU sums in row order too)
    dF, dP = diagonal(osys.F), diagonal(osys.GtG)
    assert np.array_equal(pc.diag_F.cpu().numpy(), dF) and np.array_equal(pc.diag_P.cpu().numpy(), dP)
    if kf == "chebyshev":
        assert abs(pc.inner_F.lmax - gershgorin(osys.F, dF)) <= 1e-14 * pc.inner_F.lmax
    iF = Inner(kf, sf, pc.inner_F.lmin or 0.0, pc.inner_F.lmax or 0.0)
    iP = Inner(kp, spp, pc.inner_P.lmin or 0.0, pc.inner_P.lmax or 0.0)
    v = np.random.default_rng(n).standard_normal(pc.shape[0])
    got = pc.apply(_cuda(v))
    ref = approx_schur_apply(osys.F, osys.D, osys.G, osys.GtG, osys.GtFG, v, iF, iP)
    assert _bits_equal(got, ref), rel_inf(got.cpu().numpy(), ref)
    m1 = pc.matvec(v)
    assert np.array_equal(m1, got.cpu().numpy())                      # LinearOperator surface
    m2 = pc.matvec(list(2.0 * v))                                      # staging buffers reused, results not aliased
    assert np.array_equal(m1, got.cpu().numpy()) and np.array_equal(m2, pc.apply(_cuda(2.0 * v)).cpu().numpy())


@pytest.mark.parametrize("path", [p for p in golden_files() if "n32" not in p], ids=os.path.basename)
def test_schur_apply_against_reference(path):
    """Jacobi-inner apply vs the reference composition on the reference's own matrices (1e-12)."""
    mp = _mp()
    g = load_golden(path)
    p = golden_params(g)
    bp = mp.MultiphaseBlockPreconditioner(p["n"], p["xi"], p["eta_n"], p["eta_s"])
    if golden_tables(g) is not None:
        bp.set_theta_tables(*golden_tables(g))
    A, _, F, D, G = bp.get_big_A_matrix(c=p["c"], d_u=p["d_u"])
    for nf, npp in ((1, 1), (3, 2)):
        pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("jacobi", nf),
                                          inner_P=mp.InnerSolver("jacobi", npp))
        assert rel_inf(pc.apply(_cuda(g["v"])).cpu().numpy(), g[f"schur_jacobi_{nf}_{npp}"]) <= 1e-12


def test_full_size_properties():
    """1024^2 (BASELINE configs[2]): linearity, determinism, CSR == SELL, O(h^2) consistency."""
    mp = _mp()
    n = 1024
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    assert A.nnz == 56 * n * n and F.nnz == 40 * n * n
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("chebyshev", 4),
                                      inner_P=mp.InnerSolver("chebyshev", 4))
    gen = torch.Generator(device="cuda").manual_seed(5)
    v1 = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda", generator=gen)
    v2 = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda", generator=gen)
    y1, y2 = pc.apply(v1), pc.apply(v2)
    y12 = pc.apply(2.0 * v1 - 0.5 * v2)
    assert rel_inf(y12.cpu().numpy(), (2.0 * y1 - 0.5 * y2).cpu().numpy()) <= 1e-12
    pc_csr = mp.ApproxSchurPreconditioner(F, D, G, pc.GtG, pc.GtFG, inner_F=mp.InnerSolver("chebyshev", 4),
                                          inner_P=mp.InnerSolver("chebyshev", 4), layout="csr")
    assert torch.equal(pc_csr.apply(v1), y1)                                  # CSR == SELL bit for bit
    assert torch.equal(pc.apply(v1), y1)                                      # deterministic
    # manufactured solution: ||A u - b||_inf / ||b||_inf is a truncation error, O(h^2)
    u, b = mp.manufactured_problem(n, 1.0, -1.0, 1.0, 100.0, 1.0)
    Au = A.matvec(_cuda(u)).cpu().numpy()
    assert rel_inf(Au, b) <= 1e-3
    # (the whole 1024^2 CSR is compared with the oracle bit for bit in test_gpu_configs.py)


def test_fgmres_converges_with_gpu_preconditioner():
    mp = _mp()
    n = 32
    u, b = mp.manufactured_problem(n, 1.0, -1.0, 1.0, 100.0, 1.0)
    x, info, hist = mp.solve_with_approx_schur_pc(n, 1.0, 100.0, 1.0, 1.0, -1.0, b, u,
                                                  inner_F=mp.InnerSolver("chebyshev", 8),
                                                  inner_P=mp.InnerSolver("chebyshev", 8),
                                                  tol=1e-8, maxiter=400, verbose=False)
    assert info == 0 and hist[-1] <= 1e-8 * hist[0] * 1.0001
    # discretisation error of the converged solution (velocity components), O(h^2)
    assert np.max(np.abs(x[: 4 * n * n] - u[: 4 * n * n])) < 5e-2


def test_fgmres_without_preconditioner_and_constant_theta():
    """configs[0]'s plumbing case on the GPU path: constant thn (theta_n = theta_s = 1/2), FGMRES without a
    preconditioner (solve.py:202-208) -- and the preconditioned solve cuts the iteration count."""
    mp = _mp()
    n = 16
    N = n * n
    half = np.full(N, 0.5)
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 1.0, 1.0)
    bp.set_theta_tables(half, half, half)
    A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    rng = np.random.default_rng(0)
    u = rng.standard_normal(5 * N)
    b = A.matvec(torch.from_numpy(u).cuda()).cpu().numpy()
    x, info, hist = mp.solve_without_pc(n, A, b, u, tol=1e-10, maxiter=2000, verbose=False)
    assert info == 0 and hist[-1] <= 1e-10 * hist[0] * 1.0001
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("chebyshev", 8),
                                      inner_P=mp.InnerSolver("chebyshev", 8))
    hist_pc = []
    xp, info_pc = mp.fgmres(A, torch.from_numpy(b).cuda(), M=pc, tol=1e-10, maxiter=2000, residuals=hist_pc)
    assert info_pc == 0 and len(hist_pc) < len(hist)
    # the pressure is determined up to a constant on the periodic grid: compare velocities
    assert np.max(np.abs(x[: 4 * N] - u[: 4 * N])) < 1e-6 and np.max(np.abs(xp.cpu().numpy()[: 4 * N] - u[: 4 * N])) < 1e-6


@pytest.mark.parametrize("n", [0, 1, 255, 4095, 4096, 4097, 1_000_003])
def test_exclusive_scan(n):
    """Tiled row_ptr scan (assembly / SpGEMM / extraction setup): exact against numpy, row_ptr[n] = total."""
    import ctypes
    from mp_block_preconditioners_amd._lib import check, lib, ptr, stream_handle
    rng = np.random.default_rng(n)
    cnt = torch.from_numpy(rng.integers(0, 40, size=max(n, 1)).astype(np.int32)).cuda()
    out = torch.full((n + 1,), -7, dtype=torch.int32, device="cuda")
    total = ctypes.c_int64(-1)
    check(lib().mpbp_exclusive_scan(ptr(cnt), ptr(out), n, ctypes.byref(total), stream_handle()))
    ref = np.concatenate([[0], np.cumsum(cnt.cpu().numpy()[:n], dtype=np.int64)])
    assert total.value == ref[-1]
    assert np.array_equal(out.cpu().numpy(), ref.astype(np.int32))


def test_exclusive_scan_overflow():
    import ctypes
    from mp_block_preconditioners_amd._lib import lib, ptr, stream_handle
    cnt = torch.full((5000,), 1 << 20, dtype=torch.int32, device="cuda")   # total 5.2e9 > INT32_MAX
    out = torch.empty(5001, dtype=torch.int32, device="cuda")
    total = ctypes.c_int64(0)
    rc = lib().mpbp_exclusive_scan(ptr(cnt), ptr(out), 5000, ctypes.byref(total), stream_handle())
    assert rc == -3 and b"exceed int32" in lib().mpbp_last_error()


@pytest.mark.parametrize("start_odd", [False, True])
def test_csr_wave_uniform_waves_bit_exact(start_odd):
    """k_csr_wave's uniform-wave path (64 rows of 8, 10 or 12 entries from an even start: unrolled,
    buffer-load gathers) next to waves it must not take (length 14, mixed lengths, a partial wave, an odd
    start); every epilogue mode bit-exact vs the oracle."""
    mp = _mp()
    from oracle import csr_oracle as co
    rng = np.random.default_rng(5 + start_odd)
    segs = [np.full(64, 12), np.full(64, 10), np.full(64, 8), np.full(64, 14),
            rng.integers(6, 13, size=64), np.full(64, 12), np.full(30, 12)]
    lengths = np.concatenate(([np.array([1])] if start_odd else []) + segs).astype(np.int64)
    rows = np.repeat(np.arange(lengths.size), lengths)
    cols = np.concatenate([np.sort(rng.choice(5000, size=k, replace=False)) for k in lengths])
    M = sp.csr_matrix((rng.standard_normal(rows.size), cols, np.r_[0, np.cumsum(lengths)]),
                      shape=(lengths.size, 5000))
    x, z = rng.standard_normal(5000), rng.standard_normal(lengths.size)
    dM = mp.DeviceCSR.from_scipy(M)
    for mode in (0, 1, 2):
        assert _bits_equal(dM.matvec(_cuda(x), mode=mode, z=_cuda(z)), co.spmv(M, x, z, mode=mode)), mode


def test_host_vector_length_checked():
    """The host-vector matvecs (LinearOperator surface and A @ x) reject a wrong-length vector instead of
    broadcasting it, and stay usable afterwards."""
    mp = _mp()
    bp = mp.MultiphaseBlockPreconditioner(8, 1.0, 1.0, 1.0)
    A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G)
    m = pc.shape[0]
    for bad in (np.ones(1), np.ones(m - 1), np.ones(m + 1)):
        with pytest.raises(ValueError):
            pc.approx_schur_op(bad)
        with pytest.raises(ValueError):
            pc.matvec(bad)
        with pytest.raises(ValueError):
            A @ bad
    x = np.random.default_rng(1).standard_normal(m)
    assert np.array_equal(pc.approx_schur_op(x), pc.apply(_cuda(x)).cpu().numpy())
    assert np.array_equal(A @ x, A.matvec(_cuda(x)).cpu().numpy())
    pc.release_staging()
    assert np.array_equal(pc.matvec(x), pc.apply(_cuda(x)).cpu().numpy())


@pytest.mark.parametrize("k,n", [(1, 1000), (8, 4096), (37, 100003), (151, 5000)])
def test_gram_schmidt_kernels(k, n):
    """FGMRES's projections (mpbp_gs_dot: h = V w; mpbp_gs_update: w - V^T h) against torch's fp64 GEMVs, and
    deterministic: two runs give the same bits."""
    from mp_block_preconditioners_amd._lib import check, lib, ptr, stream_handle
    g = torch.Generator(device="cuda").manual_seed(k)
    V = torch.randn(k + 3, n, dtype=torch.float64, device="cuda", generator=g)   # extra rows: only k are read
    w = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    part = torch.empty(int(lib().mpbp_gs_part_size(n, k)), dtype=torch.float64, device="cuda")
    h = torch.empty(k, dtype=torch.float64, device="cuda")
    check(lib().mpbp_gs_dot(ptr(V), n, k, ptr(w), n, ptr(part), ptr(h), stream_handle()))
    ref = V[:k] @ w
    assert float((h - ref).abs().max() / ref.abs().max()) < 1e-13
    h2 = torch.empty_like(h)
    check(lib().mpbp_gs_dot(ptr(V), n, k, ptr(w), n, ptr(part), ptr(h2), stream_handle()))
    assert torch.equal(h, h2)
    wo = torch.empty_like(w)
    check(lib().mpbp_gs_update(ptr(V), n, k, ptr(h), ptr(w), n, ptr(wo), stream_handle()))
    want = w - V[:k].T @ h
    assert float((wo - want).abs().max() / want.abs().max()) < 1e-13
    check(lib().mpbp_gs_update(ptr(V), n, k, ptr(h), ptr(w), n, ptr(w), stream_handle()))   # in place
    assert torch.equal(w, wo)
