"""Matrix-free F (rows recomputed from the thn tables) against the assembled F and the oracle.

The stencil kernels must reproduce the assembled-F sweeps bit for bit: same entry values (same
formulas and evaluation order as the assembly), summed in the same (sorted-column) order."""
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


PARAMS = [(1.0, 100.0, 1.0, 1.0, -1.0), (2.5, 1.0e4, 1.0, 0.5, -2.0), (1.0, 1.0, 1.0, 0.0, -1.0)]


@pytest.fixture(params=[0, 4, 1, 3, 8], ids=["auto", "march4", "march1", "march3", "march8"])
def stencil_kind(request):
    """Rows per workgroup of the marching kernel (kernel option march_rows): results must not depend on it."""
    from mp_block_preconditioners_amd._lib import kernel_options
    with kernel_options(march_rows=request.param):
        yield request.param


@pytest.mark.parametrize("n", [3, 4, 17, 64, 255, 300])
@pytest.mark.parametrize("prm", PARAMS, ids=["visc", "stiff", "c0"])
def test_stencil_matvec_and_sweeps_bit_exact(n, prm, stencil_kind):
    import mp_block_preconditioners_amd as mp
    from mp_block_preconditioners_amd._lib import check, lib, ptr, stream_handle
    xi, eta_n, eta_s, c, d_u = prm
    bp = mp.MultiphaseBlockPreconditioner(n, xi, eta_n, eta_s)
    _, _, F, _, _ = bp.get_big_A_matrix(c=c, d_u=d_u)
    st = F.stencil
    assert st is not None
    g = torch.Generator(device="cuda").manual_seed(n)
    x, b, d0, sub = (torch.randn(F.shape[0], dtype=torch.float64, device="cuda", generator=g) for _ in range(4))
    for mode in (0, 1, 2):
        assert _bits(st.matvec(x, mode=mode, z=b), F.matvec(x, mode=mode, z=b))
    diag = F.diagonal()
    blk = F.blocks.cstruct()
    y1, y2 = torch.empty_like(x), torch.empty_like(x)
    stencil_tabs = (ptr(st.cell), ptr(st.uface), ptr(st.vface))
    check(lib().mpbp_jacobi_step(ctypes.byref(F.cstruct()), ctypes.byref(blk), ptr(x), ptr(b), ptr(diag), ptr(sub),
                                 ptr(y1), stream_handle()))
    check(lib().mpbp_f_stencil_jacobi_step(ctypes.byref(st.prm), *stencil_tabs, None, ptr(x), ptr(b), ptr(sub), ptr(y2),
                                           stream_handle()))
    assert _bits(y1, y2)
    d1, d2 = d0.clone(), d0.clone()
    check(lib().mpbp_cheb_step(ctypes.byref(F.cstruct()), ctypes.byref(blk), ptr(x), ptr(b), ptr(diag), 0.7, 1.3,
                               ptr(d1), None, ptr(y1), stream_handle()))
    check(lib().mpbp_f_stencil_cheb_step(ctypes.byref(st.prm), *stencil_tabs, None, ptr(x), ptr(b), 0.7, 1.3, ptr(d2),
                                         None, ptr(y2), stream_handle()))
    assert _bits(y1, y2) and _bits(d1, d2)


@pytest.mark.parametrize("n", [3, 32, 96])
def test_stencil_apply_matches_assembled_and_oracle(n, stencil_kind):
    import mp_block_preconditioners_amd as mp
    from oracle.schur_oracle import Inner, approx_schur_apply
    from oracle.stokes_oracle import StokesSystem, theta_tables
    tabs = theta_tables(n)
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    bp.set_theta_tables(*tabs)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    kw = dict(inner_F=mp.InnerSolver("chebyshev", 5), inner_P=mp.InnerSolver("jacobi", 3))
    pc_st = mp.ApproxSchurPreconditioner(F, D, G, f_mode="stencil", **kw)
    pc_as = mp.ApproxSchurPreconditioner(F, D, G, pc_st.GtG, pc_st.GtFG, f_mode="assembled", **kw)
    assert pc_st.f_stencil is not None and pc_as.f_stencil is None
    v = np.random.default_rng(n).standard_normal(pc_st.shape[0])
    vt = torch.from_numpy(v).cuda()
    got = pc_st.apply(vt)
    assert torch.equal(got, pc_as.apply(vt))
    s = StokesSystem(n, 1.0, 100.0, 1.0, 1.0, -1.0, tables=tabs)
    ref = approx_schur_apply(s.F, s.D, s.G, s.GtG, s.GtFG, v, Inner("chebyshev", 5, pc_st.inner_F.lmin,
                                                                    pc_st.inner_F.lmax), Inner("jacobi", 3))
    assert _bits(got, ref), rel_inf(got.cpu().numpy(), ref)


def test_stencil_rejected_where_undefined():
    import mp_block_preconditioners_amd as mp
    bp = mp.MultiphaseBlockPreconditioner(2, 1.0, 1.0, 1.0)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    assert F.stencil is None                       # n <= 2: periodic neighbours coincide
    with pytest.raises(ValueError):
        mp.ApproxSchurPreconditioner(F, D, G, f_mode="stencil")
    pc = mp.ApproxSchurPreconditioner(F, D, G, f_mode="auto")
    assert pc.f_stencil is None


def test_graph_replay_matches_eager():
    """The apply captured into a hipGraph (bench.py's launch mode) replays to the eager result."""
    import mp_block_preconditioners_amd as mp
    bp = mp.MultiphaseBlockPreconditioner(48, 1.0, 100.0, 1.0)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G)
    v = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda")
    ref = pc.apply(v).clone()
    out = torch.zeros_like(v)
    pc.enable_profiling(8)
    g = pc.capture(v, out)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert pc.profiled_ms() == []              # no events are recorded under capture
    pc.apply(v)
    torch.cuda.synchronize()
    ms = pc.profiled_ms()
    pc.disable_profiling()
    assert len(ms) == 4 and all(t > 0 for t in ms)   # 2 solves x 2 plain sweeps (the first is fused with init)
    v.copy_(torch.randn_like(v))             # replay reads the captured buffers' new contents
    g.replay()
    assert torch.equal(out, pc.apply(v))


def _ext_local_rows(n, L, h, nf):
    """Local grid row (-h .. L+h-1) of every slot of the owned + ghost layout (RowPartition.ext_rows order)."""
    own = np.repeat(np.tile(np.arange(L), nf), n)
    above = np.repeat(np.tile(np.arange(-h, 0), nf), n)
    below = np.repeat(np.tile(np.arange(L, L + h), nf), n)
    return np.concatenate([own, above, below])


@pytest.mark.parametrize("kind", ["jacobi", "chebyshev", "spmv"])
def test_f_stencil_ghost_rows_bit_exact(kind):
    """The marching F stencil on owned + ext ghost rows (mpbp_row_part.which = 3, the CA schedule's launches):
    every computed slot equals the one-GPU result at that slot's global row, ghost rows at the periodic grid
    edge included."""
    import mp_block_preconditioners_amd as mp
    from mp_block_preconditioners_amd._lib import RowPart, check, lib, ptr, stream_handle
    from mp_block_preconditioners_amd.distributed import RowPartition
    n, h, e = 24, 4, 3
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    _, _, F, _, _ = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    st = F.stencil
    tabs = (ptr(st.cell), ptr(st.uface), ptr(st.vface))
    part = RowPartition(n, 1, 0, ghosts=True)
    gid = torch.from_numpy(part.ext_rows(4, h)).cuda()
    g = torch.Generator(device="cuda").manual_seed(3)
    x, b, d = (torch.randn(F.shape[0], dtype=torch.float64, device="cuda", generator=g) for _ in range(3))
    y = torch.empty_like(x)
    ye = torch.full((gid.numel(),), float("nan"), dtype=torch.float64, device="cuda")
    xe, be, de = x[gid].contiguous(), b[gid].contiguous(), d[gid].contiguous()
    rp = RowPart(0, n, h, 3, e, 0)
    if kind == "jacobi":
        check(lib().mpbp_f_stencil_jacobi_step(ctypes.byref(st.prm), *tabs, None, ptr(x), ptr(b), None, ptr(y),
                                               stream_handle()))
        check(lib().mpbp_f_stencil_jacobi_step(ctypes.byref(st.prm), *tabs, ctypes.byref(rp), ptr(xe), ptr(be), None,
                                               ptr(ye), stream_handle()))
    elif kind == "chebyshev":
        check(lib().mpbp_f_stencil_cheb_step(ctypes.byref(st.prm), *tabs, None, ptr(x), ptr(b), 0.7, 1.3, ptr(d),
                                             None, ptr(y), stream_handle()))
        check(lib().mpbp_f_stencil_cheb_step(ctypes.byref(st.prm), *tabs, ctypes.byref(rp), ptr(xe), ptr(be), 0.7,
                                             1.3, ptr(de), None, ptr(ye), stream_handle()))
    else:
        check(lib().mpbp_f_stencil_spmv(ctypes.byref(st.prm), *tabs, None, 1, ptr(x), ptr(b), ptr(y),
                                        stream_handle()))
        check(lib().mpbp_f_stencil_spmv(ctypes.byref(st.prm), *tabs, ctypes.byref(rp), 1, ptr(xe), ptr(be), ptr(ye),
                                        stream_handle()))
    lr = torch.from_numpy(_ext_local_rows(n, n, h, 4)).cuda()
    sel = (lr >= -e) & (lr < n + e)
    assert _bits(ye[sel], y[gid][sel])
    if kind == "chebyshev":
        assert _bits(de[sel], d[gid][sel])
    assert torch.isnan(ye[~sel]).all()     # rows beyond the ext depth are not written
