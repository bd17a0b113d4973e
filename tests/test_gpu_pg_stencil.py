"""Matrix-free D, G and Gt_G = -(D G) (rows recomputed from the cell thn table) against the assembled
operators, the sparse product and the oracle.

The pressure-side kernels must reproduce the assembled operators bit for bit: same entry values (the
assembly's formulas; for Gt_G the SpGEMM's products accumulated in D's column order, then x alpha = -1),
summed in the same sorted-column order.  The inner solves' fused first sweep (x0 = c2 b / diag recomputed
where the sweep stages x, no init pass) must equal init + sweep."""
import ctypes

import numpy as np
import pytest

from conftest import rel_inf

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(oracle_built):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _bits(a, b):
    a = a.cpu().numpy() if hasattr(a, "cpu") else np.asarray(a)
    b = b.cpu().numpy() if hasattr(b, "cpu") else np.asarray(b)
    return np.array_equal(a.view(np.uint64), b.view(np.uint64))


# (xi, eta_n, eta_s, c, d_u, d_p)
PARAMS = [(1.0, 100.0, 1.0, 1.0, -1.0, 1.0), (2.5, 1.0e4, 1.0, 0.5, -2.0, 2.5), (1.0, 1.0, 1.0, 0.0, -1.0, -0.75)]


@pytest.fixture(params=[(0, 1), (0, 0), (4, 0), (1, 0), (7, 0)], ids=["direct", "auto", "march4", "march1", "march7"])
def march_rows(request):
    """Workgroup shapes of the marching kernels, and the direct one-thread-per-cell kernel for D / G / Gt_G
    (kernel option pg_direct): results must not depend on either."""
    from mp_block_preconditioners_amd._lib import kernel_options
    rows, direct = request.param
    with kernel_options(march_rows=rows, pg_direct=direct):
        yield request.param


def _system(n, prm, tables=None):
    import mp_block_preconditioners_amd as mp
    xi, eta_n, eta_s, c, d_u, d_p = prm
    bp = mp.MultiphaseBlockPreconditioner(n, xi, eta_n, eta_s)
    if tables is not None:
        bp.set_theta_tables(*tables)
    _, _, F, D, G = bp.get_big_A_matrix(c=c, d_u=d_u, d_p=d_p)
    GtG, GtFG = bp.commutator_products(F, D, G)
    return F, D, G, GtG, GtFG


@pytest.mark.parametrize("n", [3, 4, 17, 64, 255, 300])
@pytest.mark.parametrize("prm", PARAMS, ids=["visc", "stiff", "c0-neg-dp"])
def test_pg_matvecs_and_sweeps_bit_exact(n, prm, march_rows):
    from mp_block_preconditioners_amd._lib import PG_GTG, check, lib, ptr, stream_handle
    F, D, G, GtG, _ = _system(n, prm)
    assert GtG.stencil is not None and GtG.stencil.op == PG_GTG
    g = torch.Generator(device="cuda").manual_seed(n)
    N = n * n
    for M in (D, G, GtG):
        x = torch.randn(M.shape[1], dtype=torch.float64, device="cuda", generator=g)
        z = torch.randn(M.shape[0], dtype=torch.float64, device="cuda", generator=g)
        for mode in (0, 1, 2):
            assert _bits(M.stencil.matvec(x, mode=mode, z=z), M.matvec(x, mode=mode, z=z)), (M.shape, mode)
    x, b, d0, sub = (torch.randn(N, dtype=torch.float64, device="cuda", generator=g) for _ in range(4))
    diag = GtG.diagonal()
    blk = GtG.blocks.cstruct()
    st = GtG.stencil
    for s in (None, sub):
        y1, y2 = torch.empty_like(x), torch.empty_like(x)
        check(lib().mpbp_jacobi_step(ctypes.byref(GtG.cstruct()), ctypes.byref(blk), ptr(x), ptr(b), ptr(diag), ptr(s),
                                     ptr(y1), stream_handle()))
        check(lib().mpbp_gtg_stencil_jacobi_step(ctypes.byref(st.prm), ptr(st.cell), None, ptr(x), ptr(b), ptr(s),
                                                 ptr(y2), stream_handle()))
        assert _bits(y1, y2)
        d1, d2 = d0.clone(), d0.clone()
        check(lib().mpbp_cheb_step(ctypes.byref(GtG.cstruct()), ctypes.byref(blk), ptr(x), ptr(b), ptr(diag), 0.7, 1.3,
                                   ptr(d1), ptr(s), ptr(y1), stream_handle()))
        check(lib().mpbp_gtg_stencil_cheb_step(ctypes.byref(st.prm), ptr(st.cell), None, ptr(x), ptr(b), 0.7, 1.3,
                                               ptr(d2), ptr(s), ptr(y2), stream_handle()))
        assert _bits(y1, y2) and _bits(d1, d2)


def test_pg_matches_oracle_products():
    """Gt_G from the stencil against the oracle's (-D) G on non-smooth tables (no cancellation luck)."""
    from oracle import csr_oracle as co
    from oracle.stokes_oracle import StokesSystem
    n = 20
    rng = np.random.default_rng(3)
    tabs = tuple(rng.uniform(0.05, 0.95, n * n) for _ in range(3))
    F, D, G, GtG, _ = _system(n, PARAMS[1], tabs)
    s = StokesSystem(n, 2.5, 1.0e4, 1.0, 0.5, -2.0, d_p=2.5, tables=tabs)
    x = rng.standard_normal(n * n)
    got = GtG.stencil.matvec(torch.from_numpy(x).cuda())
    assert _bits(got, co.spmv(s.GtG, x)), rel_inf(got.cpu().numpy(), co.spmv(s.GtG, x))
    xu = rng.standard_normal(4 * n * n)
    assert _bits(D.stencil.matvec(torch.from_numpy(xu).cuda()), co.spmv(s.D, xu))
    assert _bits(G.stencil.matvec(torch.from_numpy(x).cuda()), co.spmv(s.G, x))


INNERS = [(("chebyshev", 4), ("chebyshev", 3)), (("jacobi", 3), ("chebyshev", 2)), (("chebyshev", 2), ("jacobi", 4)),
          (("jacobi", 1), ("chebyshev", 1)), (("chebyshev", 5), ("jacobi", 2))]


@pytest.mark.parametrize("n", [3, 32, 97])
@pytest.mark.parametrize("inner", INNERS, ids=["c4c3", "j3c2", "c2j4", "j1c1", "c5j2"])
def test_matrix_free_apply_matches_assembled_and_oracle(n, inner):
    """Every combination of matrix-free F / D / G / Gt_G (with the fused first sweeps) equals the fully
    assembled apply and the oracle bit for bit."""
    import mp_block_preconditioners_amd as mp
    from oracle.schur_oracle import Inner, approx_schur_apply
    from oracle.stokes_oracle import StokesSystem, theta_tables
    tabs = theta_tables(n)
    F, D, G, GtG, GtFG = _system(n, PARAMS[0], tabs)
    kw = dict(inner_F=mp.InnerSolver(*inner[0]), inner_P=mp.InnerSolver(*inner[1]))
    ref_pc = mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG, f_mode="assembled", pg_mode="assembled", **kw)
    assert ref_pc.f_stencil is None and ref_pc.pg_stencil is None
    v = torch.from_numpy(np.random.default_rng(n).standard_normal(ref_pc.shape[0])).cuda()
    ref = ref_pc.apply(v)
    for f_mode in ("stencil", "assembled"):
        for pg_mode in ("stencil", "assembled"):
            pc = mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG, f_mode=f_mode, pg_mode=pg_mode, **kw)
            assert (pc.pg_stencil is not None) == (pg_mode == "stencil")
            assert torch.equal(pc.apply(v), ref), (f_mode, pg_mode)
    s = StokesSystem(n, 1.0, 100.0, 1.0, 1.0, -1.0, tables=tabs)
    iF = Inner(inner[0][0], inner[0][1], ref_pc.inner_F.lmin, ref_pc.inner_F.lmax)
    iP = Inner(inner[1][0], inner[1][1], ref_pc.inner_P.lmin, ref_pc.inner_P.lmax)
    want = approx_schur_apply(s.F, s.D, s.G, s.GtG, s.GtFG, v.cpu().numpy(), iF, iP)
    assert _bits(ref, want), rel_inf(ref.cpu().numpy(), want)


def test_pg_mode_validation():
    import mp_block_preconditioners_amd as mp
    F, D, G, GtG, GtFG = _system(8, PARAMS[0])
    with pytest.raises(ValueError):
        mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG, pg_mode="bogus")
    # a Gt_G of another grid (other d_p): auto falls back to the stored operators, "stencil" refuses
    _, _, G2, _, _ = _system(8, PARAMS[0][:5] + (2.0,))
    pc = mp.ApproxSchurPreconditioner(F, D, G2, pg_mode="auto")
    assert pc.pg_stencil is None
    with pytest.raises(ValueError):
        mp.ApproxSchurPreconditioner(F, D, G2, pg_mode="stencil")
    bp = mp.MultiphaseBlockPreconditioner(2, 1.0, 1.0, 1.0)
    _, _, F2, D2, G2 = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    assert D2.stencil is None and G2.stencil is None           # n <= 2: no matrix-free forms
    assert mp.ApproxSchurPreconditioner(F2, D2, G2).pg_stencil is None


@pytest.mark.parametrize("n", [3, 4, 5, 50, 256, 257, 300])
@pytest.mark.parametrize("prm", PARAMS, ids=["visc", "stiff", "c0-neg-dp"])
@pytest.mark.parametrize("inner", [INNERS[0], INNERS[1], INNERS[3]], ids=["c4c3", "j3c2", "j1c1"])
def test_fused_first_sweep_rebuilt_diagonal(n, prm, inner, march_rows):
    """The fused first inner sweep with the staged diagonal rebuilt from thn (k_march_init, default) equals the
    one that streams the stored diagonal (k_march<XInit>) and the fully assembled apply, bit for bit -- every
    parameter identity instance of the F policy, strips with ragged last columns (n = 257, 300), n = 3."""
    import mp_block_preconditioners_amd as mp
    F, D, G, GtG, GtFG = _system(n, prm)
    kw = dict(inner_F=mp.InnerSolver(*inner[0]), inner_P=mp.InnerSolver(*inner[1]))
    ref_pc = mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG, f_mode="assembled", pg_mode="assembled", **kw)
    pc = mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG, f_mode="stencil", pg_mode="stencil", **kw)
    v = torch.from_numpy(np.random.default_rng(n + 7).standard_normal(ref_pc.shape[0])).cuda()
    ref = ref_pc.apply(v)
    for mode in (1, 0):
        pc.set_kernel_opts(init_diag=mode)
        assert _bits(pc.apply(v), ref), (mode, rel_inf(pc.apply(v).cpu().numpy(), ref.cpu().numpy()))


@pytest.mark.parametrize("n", [3, 4, 5, 64, 257])
@pytest.mark.parametrize("prm", PARAMS, ids=["visc", "stiff", "c0-neg-dp"])
@pytest.mark.parametrize("sweeps", [2, 3, 4, 5])
def test_second_f_solve_recomputes_g(n, prm, sweeps, march_rows):
    """The second F solve with W = G x_p recomputed inside its sweeps (plan.fuse_g: no G launch) equals the
    unfused apply (G kernel, then the sweeps reading W) bit for bit: first sweep (staged x0 = c2 W / diag) and
    the plain sweeps, every parameter identity instance, the periodic edges, ragged strips (n = 257)."""
    import mp_block_preconditioners_amd as mp
    F, D, G, GtG, GtFG = _system(n, prm)
    kw = dict(inner_F=mp.InnerSolver("chebyshev", sweeps), inner_P=mp.InnerSolver("chebyshev", 3))
    fused = mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG, **kw)
    plain = mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG, fuse_g=False, **kw)
    assert fused.fuse_g and not plain.fuse_g
    v = torch.from_numpy(np.random.default_rng(n + sweeps).standard_normal(fused.shape[0])).cuda()
    a, b = fused.apply(v), plain.apply(v)
    assert _bits(a, b), rel_inf(a.cpu().numpy(), b.cpu().numpy())
    # Jacobi F solves keep the G launch
    assert not mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG, inner_F=mp.InnerSolver("jacobi", 3)).fuse_g
