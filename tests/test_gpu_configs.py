"""Every BASELINE.json config through the product path (HIP kernels via the C ABI) against the oracle.

configs[0]  32 x 32, constant thn (the reference's 0.75 case, solve.py:60-68): GPU assembly bit-exact vs the
            oracle and within 1e-12 of the reference's fixture; the GPU preconditioner as the M of scipy's
            GMRES on the host CSR (the LinearOperator drop-in, solve.py:279-285).
configs[1]  256 x 256 variable thn, the bench's default apply (matrix-free F / D / G / Gt_G marching kernels,
            SELL Gt_F_G, Chebyshev-4 inner solves), bit-exact vs oracle/schur_oracle.py; hipGraph replay too.
configs[2]  1024 x 1024: the whole CSR assembly (A, F, D, G) bit-exact vs oracle/stokes_oracle.py.
configs[3]  eta_n / eta_s = 1e4 with Chebyshev inner sweeps: bit-exact vs the oracle at 256^2; at 1024^2
            linearity, determinism, CSR == SELL and matrix-free == assembled F, bit for bit.
configs[4]  (2048^2 over 8 GPUs) is the driver's multi-GPU bench; its partitioned apply is covered by
            tests/test_gpu_distributed.py (and bench.py's bit_exact_vs_single_gpu).
"""
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


def _cuda(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()


def _bits_equal(a, b):
    a = a.cpu().numpy() if hasattr(a, "cpu") else np.asarray(a)
    return np.array_equal(np.asarray(a, dtype=np.float64).view(np.uint64), np.asarray(b, dtype=np.float64).view(np.uint64))


def _same_csr(dev, ref):
    got = dev.to_scipy()
    ref = sp.csr_matrix(ref)
    assert got.shape == ref.shape
    assert np.array_equal(got.indptr, ref.indptr), "row_ptr differs"
    assert np.array_equal(got.indices, ref.indices), "col_idx differs"
    assert np.array_equal(got.data.view(np.uint64), ref.data.view(np.uint64)), \
        f"values differ (max {np.max(np.abs(got.data - ref.data)):.3e})"


def _gpu_system(n, xi, eta_n, eta_s, tables, c=1.0, d_u=-1.0):
    mp = _mp()
    bp = mp.MultiphaseBlockPreconditioner(n, xi, eta_n, eta_s)
    bp.set_theta_tables(*tables)
    return bp, bp.get_big_A_matrix(c=c, d_u=d_u)


def _oracle_apply(pc, osys, v, kf, sf, kp, spp):
    from oracle.schur_oracle import Inner, approx_schur_apply
    iF = Inner(kf, sf, pc.inner_F.lmin or 0.0, pc.inner_F.lmax or 0.0)
    iP = Inner(kp, spp, pc.inner_P.lmin or 0.0, pc.inner_P.lmax or 0.0)
    return approx_schur_apply(osys.F, osys.D, osys.G, osys.GtG, osys.GtFG, v, iF, iP)


# ---- configs[0] ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("path", [p for p in golden_files() if "const75" in p], ids=lambda p: p.split("/")[-1])
def test_config0_constant_theta_assembly(path):
    """Constant-thn GPU assembly: bit-exact vs the oracle on the same tables, 1e-12 vs the reference."""
    from oracle import csr_oracle as co
    from oracle.stokes_oracle import StokesSystem
    from test_oracle_golden import assert_matrix_matches
    g = load_golden(path)
    p = golden_params(g)
    tabs = golden_tables(g)
    bp, (A, _, F, D, G) = _gpu_system(p["n"], p["xi"], p["eta_n"], p["eta_s"], tabs, p["c"], p["d_u"])
    osys = StokesSystem(**p, tables=tabs, products=True)
    for dev, ref in ((A, osys.A), (F, osys.F), (D, osys.D), (G, osys.G)):
        _same_csr(dev, ref)
    assert_matrix_matches(A.to_scipy(), golden_csr(g, "A"))
    Au = A.matvec(_cuda(g["u_vec"])).cpu().numpy()
    assert _bits_equal(Au, co.spmv(osys.A, g["u_vec"])) and rel_inf(Au, g["Au"]) <= 1e-12   # apply.py:72
    GtG, GtFG = bp.commutator_products(F, D, G)
    _same_csr(GtG, osys.GtG)
    _same_csr(GtFG, osys.GtFG)
    if "F_data" in g:
        assert_matrix_matches(GtFG.to_scipy(), golden_csr(g, "GtFG"))


def test_config0_gpu_preconditioner_in_scipy_gmres():
    """configs[0] plumbing with the GPU apply as the drop-in M of scipy's GMRES on the host CSR A (the
    reference drives a LinearOperator from a host Krylov loop, solve.py:279-285)."""
    import scipy.sparse.linalg as spla
    mp = _mp()
    n = 32
    _, (A, _, F, D, G) = _gpu_system(n, 1.0, 1.0, 1.0, (0.75, 0.75, 0.75))
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("chebyshev", 8),
                                      inner_P=mp.InnerSolver("chebyshev", 8))
    Ah = A.to_scipy()
    u, b = mp.manufactured_problem_constant(n, 1.0, -1.0, 1.0, 1.0, 1.0, theta=0.75)
    x, info = spla.gmres(Ah, b, M=pc, rtol=1e-10, restart=300, maxiter=3)
    assert info == 0
    N4 = 4 * n * n
    assert np.max(np.abs(x[:N4] - u[:N4])) < 2e-2                     # O(h^2) discretisation error
    calls = {"pc": 0, "none": 0}

    def counted(key):
        def mv(v):
            calls[key] += 1
            return Ah @ v
        return spla.LinearOperator(Ah.shape, matvec=mv, dtype=np.float64)
    r = np.random.default_rng(0).standard_normal(Ah.shape[0])
    r[N4:] -= r[N4:].mean()
    _, i1 = spla.gmres(counted("pc"), r, M=pc, rtol=1e-8, restart=500, maxiter=3)
    _, i2 = spla.gmres(counted("none"), r, rtol=1e-8, restart=500, maxiter=3)
    assert i1 == 0 and calls["pc"] < calls["none"], calls


# ---- configs[1] and configs[3] at 256^2: the bench's apply vs the oracle, bit for bit ------------------------
CFG_256 = [("config1", 1.0, 100.0, 1.0, ("chebyshev", 4, "chebyshev", 4)),
           ("config3_stiff", 1.0, 1.0e4, 1.0, ("chebyshev", 4, "chebyshev", 4)),
           ("config3_stiff_cheb8", 1.0, 1.0e4, 1.0, ("chebyshev", 8, "chebyshev", 6))]


@pytest.fixture(scope="module")
def oracle_256():
    from oracle.stokes_oracle import StokesSystem, theta_tables
    tabs = theta_tables(256)
    cache = {}

    def get(xi, eta_n, eta_s):
        key = (xi, eta_n, eta_s)
        if key not in cache:
            cache[key] = StokesSystem(256, xi, eta_n, eta_s, 1.0, -1.0, tables=tabs)
        return tabs, cache[key]
    return get


@pytest.mark.parametrize("layout", ["sell", "csr"])
@pytest.mark.parametrize("cfg", CFG_256, ids=[c[0] for c in CFG_256])
def test_256_apply_bit_exact_vs_oracle(cfg, layout, oracle_256):
    mp = _mp()
    _, xi, eta_n, eta_s, (kf, sf, kp, spp) = cfg
    tabs, osys = oracle_256(xi, eta_n, eta_s)
    _, (_, _, F, D, G) = _gpu_system(256, xi, eta_n, eta_s, tabs)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver(kf, sf), inner_P=mp.InnerSolver(kp, spp),
                                      layout=layout)
    assert pc.f_stencil is not None and pc.pg_stencil is not None     # the bench's matrix-free operators
    _same_csr(pc.GtG, osys.GtG)
    _same_csr(pc.GtFG, osys.GtFG)
    v = np.random.default_rng(256).standard_normal(pc.shape[0])
    got = pc.apply(_cuda(v))
    ref = _oracle_apply(pc, osys, v, kf, sf, kp, spp)
    assert _bits_equal(got, ref), rel_inf(got.cpu().numpy(), ref)
    if layout == "sell":   # the bench's launch mode: the captured apply replays to the same bits
        vt, out = _cuda(v), torch.zeros(pc.shape[0], dtype=torch.float64, device="cuda")
        g = pc.capture(vt, out)
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert _bits_equal(out, ref)


# ---- configs[2]: the full 1024^2 assembly -------------------------------------------------------------------
def test_1024_assembly_bit_exact_vs_oracle():
    """A, F, D, G at the headline size against the oracle's vectorised assembly on the same thn tables."""
    from oracle.stokes_oracle import StokesSystem, theta_tables
    n = 1024
    tabs = theta_tables(n)
    osys = StokesSystem(n, 1.0, 100.0, 1.0, 1.0, -1.0, tables=tabs, products=False)
    _, (A, _, F, D, G) = _gpu_system(n, 1.0, 100.0, 1.0, tabs)
    assert A.nnz == 56 * n * n and F.nnz == 40 * n * n
    for dev, ref in ((A, osys.A), (F, osys.F), (D, osys.D), (G, osys.G)):
        _same_csr(dev, ref)


# ---- configs[3] at 1024^2: size-independent properties -----------------------------------------------------
def test_1024_stiff_properties():
    mp = _mp()
    n = 1024
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 1.0e4, 1.0)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    iF, iP = mp.InnerSolver("chebyshev", 4), mp.InnerSolver("chebyshev", 4)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP)
    gen = torch.Generator(device="cuda").manual_seed(7)
    v1 = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda", generator=gen)
    v2 = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda", generator=gen)
    y1, y2 = pc.apply(v1).clone(), pc.apply(v2).clone()
    y12 = pc.apply(2.0 * v1 - 0.5 * v2)
    assert rel_inf(y12.cpu().numpy(), (2.0 * y1 - 0.5 * y2).cpu().numpy()) <= 1e-12      # linearity
    assert torch.equal(pc.apply(v1), y1)                                                  # determinism
    pc_csr = mp.ApproxSchurPreconditioner(F, D, G, pc.GtG, pc.GtFG, inner_F=iF, inner_P=iP, layout="csr")
    assert torch.equal(pc_csr.apply(v1), y1)                                              # CSR == SELL
    del pc_csr
    pc_asm = mp.ApproxSchurPreconditioner(F, D, G, pc.GtG, pc.GtFG, inner_F=iF, inner_P=iP, f_mode="assembled",
                                          pg_mode="assembled")
    assert torch.equal(pc_asm.apply(v1), y1)                                              # matrix-free == assembled


# ---- configs[2] with the multigrid inner solves (the bench's mg:1 / mg:1 apply) at 1024^2 ----------------------
def test_1024_mg_apply_properties():
    """The headline-size Schur apply with V(2,2) multigrid inner solves: linear (1e-12), deterministic, hipGraph
    replay == eager, and every kernel choice the library makes for a level (stencil-values / SELL on the large
    coarse levels, grouped / SELL on the small ones, matrix-free / stored transfers) gives the same bits -- the
    256^2 oracle tests (tests/test_gpu_mg.py) pin those choices against oracle/mg_oracle.py."""
    mp = _mp()
    from mp_block_preconditioners_amd._lib import check, lib
    n = 1024
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("mg", 1), inner_P=mp.InnerSolver("mg", 1))
    gen = torch.Generator(device="cuda").manual_seed(11)
    v1 = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda", generator=gen)
    v2 = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda", generator=gen)
    y1, y2 = pc.apply(v1).clone(), pc.apply(v2).clone()
    y12 = pc.apply(2.0 * v1 - 0.5 * v2)
    # linearity: ~200 launches with the coarsest pseudo-inverses between them (2.4e-12 measured; before mg.COARSE_RCOND
    # the pressure solve's inverted roundoff mode made this 0.096)
    assert rel_inf(y12.cpu().numpy(), (2.0 * y1 - 0.5 * y2).cpu().numpy()) <= 1e-10
    assert torch.equal(pc.apply(v1), y1)                                                  # determinism
    assert y1.abs().max().item() < 1e6, "the pressure solve inverted its null space"
    out = torch.empty_like(v1)
    g = pc.capture(v1, out)
    g.replay()
    torch.cuda.synchronize()
    y1h = y1.cpu().numpy()
    assert _bits_equal(out, y1h)                                                          # graph == eager
    for opt in ("mg_svl", "mg_group_rows", "mg_mf_transfer"):   # cumulative, as each kernel form is switched off
        pc.set_kernel_opts(**{opt: 0})
        assert _bits_equal(pc.apply(v1), y1h), opt
