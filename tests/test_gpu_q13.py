"""Gt_F_G in the 13-point diamond layout (values only, columns implicit in the grid): the SpMV against the
sequential C oracle's CSR SpMV of the same product, bit for bit, including the cells whose diamond wraps
around the periodic edges (their products are summed in wrapped-column order), and the full apply with the
diamond layout against the assembled one."""
import ctypes

import numpy as np
import pytest

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


PARAMS = [(1.0, 100.0, 1.0, 1.0, -1.0, 1.0), (2.5, 1.0e4, 1.0, 0.5, -2.0, 2.5)]


def _mp():
    import mp_block_preconditioners_amd as mp
    return mp


def _rel(a, b):
    a, b = a.cpu().numpy(), b.cpu().numpy()
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


def _products(n, prm):
    import mp_block_preconditioners_amd as mp
    xi, eta_n, eta_s, c, d_u, d_p = prm
    bp = mp.MultiphaseBlockPreconditioner(n, xi, eta_n, eta_s)
    _, _, F, D, G = bp.get_big_A_matrix(c=c, d_u=d_u, d_p=d_p)
    GtG, GtFG = bp.commutator_products(F, D, G)
    return F, D, G, GtG, GtFG


@pytest.mark.parametrize("n", [5, 6, 7, 16, 64, 257, 300])
@pytest.mark.parametrize("prm", PARAMS, ids=["visc", "stiff"])
def test_q13_spmv_matches_oracle(n, prm):
    from mp_block_preconditioners_amd import _lib
    from mp_block_preconditioners_amd._lib import check, lib, ptr, stream_handle
    from oracle import csr_oracle as co
    *_, GtFG = _products(n, prm)
    Q = GtFG.to_scipy()
    assert np.all(np.diff(Q.indptr) == 13)
    vals = torch.empty(13 * n * n, dtype=torch.float64, device="cuda")
    check(lib().mpbp_q13_build(ctypes.byref(GtFG.cstruct()), n, ptr(vals), stream_handle()))
    rng = np.random.default_rng(n)
    x, z = rng.standard_normal(n * n), rng.standard_normal(n * n)
    xt, zt = torch.from_numpy(x).cuda(), torch.from_numpy(z).cuda()
    want = co.spmv(Q, x)
    for mode, ref in ((_lib.SPMV_STORE, want), (_lib.SPMV_ADD, co.spmv(Q, x, z, 1)),
                      (_lib.SPMV_RESID, co.spmv(Q, x, z, 2))):
        y = torch.full((n * n,), np.nan, dtype=torch.float64, device="cuda")
        check(lib().mpbp_q13_spmv(n, ptr(vals), mode, ptr(xt), ptr(zt), ptr(y), stream_handle()))
        assert _bits(y, ref), (mode, float(np.max(np.abs(y.cpu().numpy() - ref))))


def test_q13_rejects_other_patterns():
    import mp_block_preconditioners_amd as mp
    from mp_block_preconditioners_amd._lib import MpbpError, check, lib, ptr, stream_handle
    F, D, G, GtG, GtFG = _products(8, PARAMS[0])
    vals = torch.empty(13 * 64, dtype=torch.float64, device="cuda")
    with pytest.raises(MpbpError, match="diamond"):   # Gt_G is the 5-point stencil
        check(lib().mpbp_q13_build(ctypes.byref(GtG.cstruct()), 8, ptr(vals), stream_handle()))
    with pytest.raises(ValueError):
        mp.ApproxSchurPreconditioner(F, D, G, GtG, GtG, q_mode="diamond")
    assert mp.ApproxSchurPreconditioner(F, D, G, GtG, GtG, q_mode="auto").q13 is None
    assert mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG).q13 is not None
    F4, D4, G4, GtG4, GtFG4 = _products(4, PARAMS[0])
    assert mp.ApproxSchurPreconditioner(F4, D4, G4, GtG4, GtFG4).q13 is None   # n < 5: assembled


@pytest.mark.parametrize("n", [5, 33, 256])
@pytest.mark.parametrize("layout", ["sell", "csr"])
def test_apply_with_diamond_matches_assembled(n, layout):
    import mp_block_preconditioners_amd as mp
    F, D, G, GtG, GtFG = _products(n, PARAMS[0])
    kw = dict(inner_F=mp.InnerSolver("chebyshev", 4), inner_P=mp.InnerSolver("chebyshev", 4), layout=layout)
    a = mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG, q_mode="assembled", **kw)
    b = mp.ApproxSchurPreconditioner(F, D, G, GtG, GtFG, q_mode="diamond", **kw)
    assert a.q13 is None and b.q13 is not None
    v = torch.from_numpy(np.random.default_rng(3).standard_normal(a.shape[0])).cuda()
    assert _bits(a.apply(v), b.apply(v))


@pytest.mark.parametrize("n", [36, 64, 100, 256])
@pytest.mark.parametrize("prm", [(1.0, 100.0, 1.0, 1.0, -1.0), (1.0, 1.0e4, 1.0, 1.0, -1.0), (2.5, 3.0, 0.5, 0.7, -2.0)],
                         ids=["visc", "stiff", "general"])
def test_gtfg_matrix_free_product(n, prm):
    """Kernel option q13_mf (tolerance mode, one GPU): x_b = Gt_F_G x_a applied as -(D (F (G x_a))) on tiles (k_qmf)
    instead of the stored product: the apply stays within north_star's 1e-12 relative inf-norm of the stored-product
    apply and of the exact (oracle-identical) apply, and its hipGraph replay equals the eager apply bit for bit."""
    xi, eta_n, eta_s, c, d_u = prm
    mp = _mp()
    bp = mp.MultiphaseBlockPreconditioner(n, xi, eta_n, eta_s)
    _, _, F, D, G = bp.get_big_A_matrix(c=c, d_u=d_u)
    kw = dict(inner_F=mp.InnerSolver("chebyshev", 4), inner_P=mp.InnerSolver("chebyshev", 4))
    fast = mp.ApproxSchurPreconditioner(F, D, G, numerics="fast", **kw)
    exact = mp.ApproxSchurPreconditioner(F, D, G, fast.GtG, fast.GtFG, **kw)
    v = torch.randn(fast.shape[0], dtype=torch.float64, device="cuda",
                    generator=torch.Generator(device="cuda").manual_seed(n + 3))
    fast.set_kernel_opts(q13_mf=0)
    stored = fast.apply(v).clone()
    fast.set_kernel_opts(q13_mf=1)
    mf = fast.apply(v).clone()
    e_stored = _rel(mf, stored)
    e_exact = _rel(mf, exact.apply(v))
    print(f"q13_mf n={n} {prm}: vs stored {e_stored:.3e}, vs exact {e_exact:.3e}")
    assert 0.0 < e_stored <= 1e-12 and e_exact <= 1e-12, (e_stored, e_exact)
    out = torch.empty_like(v)
    g = fast.capture(v, out)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, mf)
