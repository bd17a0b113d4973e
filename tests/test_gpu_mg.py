"""Geometric multigrid inner solves (mg.py, mpbp_mg_*) against oracle/mg_oracle.py, bit for bit.

The reference's inner inverses are ILUT (solve.py:250-254) and its comments name multigrid as the scalable
choice (solve.py:266, 274); the cycle itself has no reference counterpart, so these tests pin the GPU to the
CPU restatement (transfers, Galerkin coarse operators, V-cycles, the Schur apply with multigrid inner solves),
and check the solve-level effect: FGMRES iterations drop against the 4-sweep Chebyshev inner solves.
"""
import numpy as np
import pytest
import scipy.sparse as sp

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


def _bits(a):
    a = a.cpu().numpy() if hasattr(a, "cpu") else np.asarray(a)
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def _same_csr(dev, ref):
    got = dev.to_scipy()
    ref = sp.csr_matrix(ref)
    assert got.shape == ref.shape
    assert np.array_equal(got.indptr, ref.indptr), "row_ptr differs"
    assert np.array_equal(got.indices, ref.indices), "col_idx differs"
    assert np.array_equal(got.data.view(np.uint64), ref.data.view(np.uint64)), "values differ"


def _system(n, eta_n=100.0, eta_s=1.0):
    from oracle.stokes_oracle import StokesSystem, theta_tables
    mp = _mp()
    tables = theta_tables(n)
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, eta_n, eta_s)
    bp.set_theta_tables(*tables)
    A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    return bp, (A, F, D, G), StokesSystem(n, 1.0, eta_n, eta_s, tables=tables)


@pytest.mark.parametrize("n", [4, 8, 16, 64])
@pytest.mark.parametrize("which", ["P", "R"])
def test_transfer_bit_exact(n, which):
    mp = _mp()
    from mp_block_preconditioners_amd import _lib
    from mp_block_preconditioners_amd.mg import transfer
    from oracle import mg_oracle as mo
    for fields in (mp.FIELDS_PRESSURE, mp.FIELDS_VELOCITY):
        got = transfer(n, fields, _lib.MG_P if which == "P" else _lib.MG_R, torch.device("cuda"))
        _same_csr(got, mo.transfer(n, fields, which))


def test_transfer_rejects_bad_grids():
    from mp_block_preconditioners_amd import _lib
    from mp_block_preconditioners_amd.mg import transfer
    for n in (2, 7):
        with pytest.raises(_lib.MpbpError):
            transfer(n, ((0, 0),), _lib.MG_P, torch.device("cuda"))


@pytest.mark.parametrize("coarsest", [8, 16])
@pytest.mark.parametrize("n", [16, 32])
def test_hierarchy_bit_exact(n, coarsest):
    """Galerkin levels, transfers and smoothing bounds vs the oracle (coarsening stops at n <= coarsest, but
    happens at least once: n = 16 with coarsest 16 still has the 8^2 level)."""
    mp = _mp()
    from oracle import mg_oracle as mo
    from oracle.schur_oracle import gershgorin
    _, (A, F, D, G), S = _system(n)
    GtG, _ = mp.MultiphaseBlockPreconditioner.commutator_products(F, D, G)
    for M, Mh, fields in ((F, S.F, mp.FIELDS_VELOCITY), (GtG, S.GtG, mp.FIELDS_PRESSURE)):
        mg = mp.Multigrid(M, n, fields, coarsest=coarsest)
        ops, Ps, Rs = mo.hierarchy(Mh, n, fields, coarsest)
        assert len(ops) >= 2
        assert mg.sizes == [m for _, m in ops]
        for l, (Ml, _) in enumerate(ops):
            _same_csr(mg.ops[l], Ml)
            lmax = mg.bounds[l][1]
            ref = gershgorin(Ml, np.asarray(Ml.diagonal()))
            assert abs(lmax - ref) <= 1e-12 * ref
        for l in range(len(Ps)):
            _same_csr(mg.P[l], Ps[l])
            _same_csr(mg.R[l], Rs[l])


@pytest.fixture(params=[65536, 0], ids=["grp", "nogrp"])
def group_rows(request):
    """Small multigrid levels on the grouped CSR kernel (default threshold) or on the SELL / CSR row kernels."""
    from mp_block_preconditioners_amd._lib import kernel_options
    with kernel_options(mg_group_rows=request.param):
        yield request.param


@pytest.fixture(params=[1, 0], ids=["mftransfer", "storedtransfer"])
def mf_transfer(request):
    """Whole-grid transfers matrix-free (default) or from their stored CSR / SELL / grouped forms."""
    from mp_block_preconditioners_amd._lib import kernel_options
    with kernel_options(mg_mf_transfer=request.param):
        yield request.param


@pytest.fixture(params=[1, 0], ids=["fusesmall", "nofusesmall"])
def fuse_small(request):
    """Small grouped levels' residual + restriction as one launch (k_grp_rr; default) or as two."""
    from mp_block_preconditioners_amd._lib import kernel_options
    with kernel_options(mg_fuse_small=request.param):
        yield request.param


@pytest.fixture(params=[False, True], ids=["rowlayouts", "svl"])
def svl_all(request, monkeypatch):
    """Every coarse level with a stencil-values copy (mg.SVL_MIN_ROWS = 0), or the default (none at these sizes)."""
    from mp_block_preconditioners_amd import mg
    if request.param:
        monkeypatch.setattr(mg, "SVL_MIN_ROWS", 0)
    return request.param


@pytest.mark.parametrize("n", [16, 64])
def test_stencil_values_spmv_bit_exact(n):
    """The stencil-values layout of every coarse Galerkin level (F: 4 fields, 40 / 46 entries per row; Gt_G: 21 / 25)
    against the oracle's sequential CSR sums, every mode; interior rows from the layout, edge rows from the CSR."""
    mp = _mp()
    from oracle import csr_oracle as co
    from mp_block_preconditioners_amd.mg import StencilValues
    _, (A, F, D, G), S = _system(n)
    GtG, _ = mp.MultiphaseBlockPreconditioner.commutator_products(F, D, G)
    rng = np.random.default_rng(7 + n)
    built = 0
    for M, fields in ((F, mp.FIELDS_VELOCITY), (GtG, mp.FIELDS_PRESSURE)):
        mg = mp.Multigrid(M, n, fields, svl_min_rows=None)
        for l in range(1, mg.nlevels):
            V = StencilValues.build(mg.ops[l], len(fields), mg.sizes[l])
            if mg.sizes[l] < 16 and V is None:   # (too small for the stencil's reach: the SELL / CSR forms serve it)
                continue
            assert V is not None, (len(fields), mg.sizes[l])
            built += 1
            assert V.edge_rows.numel() == len(fields) * (mg.sizes[l] ** 2 - (mg.sizes[l] - 2 * V.reach) ** 2)
            Mh = mg.ops[l].to_scipy()
            x = rng.standard_normal(Mh.shape[1])
            z = rng.standard_normal(Mh.shape[0])
            for mode in (0, 1, 2):
                got = V.matvec(_cuda(x), mode=mode, z=_cuda(z))
                assert np.array_equal(_bits(got), _bits(co.spmv(Mh, x, z, mode=mode))), (l, mode)
            # the smoothing sweep (mpbp_svl_cheb_step) == the CSR sweep, every output
            import ctypes
            from mp_block_preconditioners_amd._lib import check, lib, ptr, stream_handle
            M, dg = mg.ops[l], mg.diags[l]
            xd, bd = _cuda(x), _cuda(z)
            outs = []
            for fn in ("svl", "csr"):
                d = _cuda(np.linspace(-1.0, 1.0, M.shape[0]))
                xo = torch.empty_like(d)
                if fn == "svl":
                    check(lib().mpbp_svl_cheb_step(ctypes.byref(V.cstruct()), ctypes.byref(M.cstruct()), ptr(xd),
                                                   ptr(bd), ptr(dg), 0.3, 0.7, ptr(d), None, ptr(xo), stream_handle()))
                else:
                    check(lib().mpbp_cheb_step(ctypes.byref(M.cstruct()), ctypes.byref(M.blocks.cstruct()), ptr(xd),
                                               ptr(bd), ptr(dg), 0.3, 0.7, ptr(d), None, ptr(xo), stream_handle()))
                outs.append((_bits(d), _bits(xo)))
            assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    assert built >= 2
    # not of the form: a non-uniform operator is refused
    assert StencilValues.build(A, 5, n) is None


@pytest.mark.parametrize("sell", [True, False], ids=["sell", "csr"])
@pytest.mark.parametrize("n,cycles,pre,post", [(16, 1, 2, 2), (32, 2, 2, 2), (64, 1, 1, 3), (64, 3, 2, 1)])
def test_mg_solve_bit_exact(n, cycles, pre, post, sell, group_rows, svl_all, mf_transfer, fuse_small):
    """V-cycles vs the oracle: with the SELL-64 copies of every level and the dense coarse kernel (default), and
    with the CSR forms throughout; the small levels and transfers on the grouped CSR kernel (several lanes per row,
    the row's sum in order) or on the row kernels; the small grouped levels' residual + restriction in one launch
    (mg_fuse_small) or in two."""
    mp = _mp()
    from oracle import mg_oracle as mo
    _, (A, F, D, G), S = _system(n)
    GtG, _ = mp.MultiphaseBlockPreconditioner.commutator_products(F, D, G)
    rng = np.random.default_rng(n + cycles)
    for M, Mh, fields in ((F, S.F, mp.FIELDS_VELOCITY), (GtG, S.GtG, mp.FIELDS_PRESSURE)):
        mg = mp.Multigrid(M, n, fields, pre=pre, post=post, cycles=cycles, sell=sell)
        assert (mg.coarse_dense is not None) == sell and (mg.sells[0][1] is not None) == sell
        ora = mo.MgOracle(Mh, n, fields, pre=pre, post=post, cycles=cycles, bounds=mg.bounds,
                          coarse_inv=mg.coarse_inv_host)
        b = rng.standard_normal(M.shape[0])
        sub = rng.standard_normal(M.shape[0])
        got = mg.solve(_cuda(b))
        assert np.array_equal(_bits(got), _bits(ora.solve(b)))
        got_s = mg.solve(_cuda(b), sub=_cuda(sub))
        assert np.array_equal(_bits(got_s), _bits(ora.solve(b, sub=sub)))


def test_mg_reduces_residual():
    """One V-cycle is a contraction on F and Gt_G at 128^2 (rates well below the Chebyshev-4 sweeps')."""
    mp = _mp()
    n = 128
    _, (A, F, D, G), _ = _system(n)
    GtG, _ = mp.MultiphaseBlockPreconditioner.commutator_products(F, D, G)
    gen = torch.Generator(device="cuda").manual_seed(5)
    for M, fields in ((F, mp.FIELDS_VELOCITY), (GtG, mp.FIELDS_PRESSURE)):
        mg = mp.Multigrid(M, n, fields)
        xt = torch.randn(M.shape[0], dtype=torch.float64, device="cuda", generator=gen)
        b = M.matvec(xt)
        x = torch.zeros_like(b)
        r0 = float(torch.linalg.vector_norm(b))
        for _ in range(4):
            x = x + mg.solve(b - M.matvec(x))
        rate = (float(torch.linalg.vector_norm(b - M.matvec(x))) / r0) ** 0.25
        assert rate < 0.2, rate


def _oracle_mg_apply(S, pc, v):
    """approx_schur_op (solve.py:257-277) with the multigrid oracle as both inner inverses."""
    from oracle import csr_oracle as co
    from oracle import mg_oracle as mo
    mF, mP = pc.mg_F, pc.mg_P
    oF = mo.MgOracle(S.F, mF.n, mF.fields, mF.pre, mF.post, mF.cycles, bounds=mF.bounds,
                     coarse_inv=mF.coarse_inv_host, coarsest=mF.coarsest)
    oP = mo.MgOracle(S.GtG, mP.n, mP.fields, mP.pre, mP.post, mP.cycles, bounds=mP.bounds,
                     coarse_inv=mP.coarse_inv_host, coarsest=mP.coarsest)
    nu = S.F.shape[0]
    Finv_v = oF.solve(v[:nu])
    rhs = co.spmv(S.D, Finv_v, v[nu:], mode=1)
    x_a = oP.solve(rhs)
    x_b = co.spmv(S.GtFG, x_a)
    x_p = oP.solve(x_b)
    u = oF.solve(co.spmv(S.G, x_p), sub=Finv_v)
    return np.concatenate([u, x_p])


@pytest.mark.parametrize("n", [16, 64])
@pytest.mark.parametrize("pre", [2, 3, 1])
@pytest.mark.parametrize("layout,f_mode,pg_mode", [("sell", "auto", "auto"), ("csr", "assembled", "assembled")])
def test_schur_apply_mg_bit_exact(n, layout, f_mode, pg_mode, pre, group_rows, svl_all):
    """The Schur apply with multigrid inner solves vs the oracle; with matrix-free level-0 operators the first
    pre-smoothing sweep stages its x0 itself (no init launch) -- pre = 2, 3 take that path, pre = 1 the init."""
    mp = _mp()
    _, (A, F, D, G), S = _system(n)
    inner = mp.InnerSolver("mg", 1, pre=pre)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=inner, inner_P=mp.InnerSolver("mg", 2, pre=pre), layout=layout,
                                      f_mode=f_mode, pg_mode=pg_mode)
    if f_mode == "auto":
        assert pc.f_stencil is not None and pc.pg_stencil is not None   # level 0 runs matrix-free
    v = np.random.default_rng(n).standard_normal(pc.shape[0])
    got = pc.apply(_cuda(v))
    ref = _oracle_mg_apply(S, pc, v)
    assert np.array_equal(_bits(got), _bits(ref))
    # hipGraph replay == eager
    vd, out = _cuda(v), torch.empty(pc.shape[0], dtype=torch.float64, device="cuda")
    g = pc.capture(vd, out)
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(_bits(out), _bits(ref))


def test_fgmres_iterations_drop_with_mg():
    """configs[1]-style solve at 64^2 (eta_n = 100): the 4-sweep Chebyshev inner solves leave FGMRES short of
    1e-8 in the reference's 150 iterations; one V-cycle per inner solve gets there in well under 100."""
    mp = _mp()
    n = 64
    _, (A, F, D, G), _ = _system(n)
    u, b = mp.manufactured_problem(n, etan=100.0, etas=1.0)
    bd = _cuda(b)
    its = {}
    for name, iF, iP in (("cheb4", mp.InnerSolver("chebyshev", 4), mp.InnerSolver("chebyshev", 4)),
                         ("mg", mp.InnerSolver("mg", 1), mp.InnerSolver("mg", 1))):
        pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP)
        hist = []
        x, info = mp.fgmres(A, bd, M=pc, tol=1e-8, maxiter=150, residuals=hist)
        its[name] = (len(hist) - 1, info)
        if name == "mg":
            assert info == 0
            err = np.max(np.abs(x.cpu().numpy()[: 4 * n * n] - u[: 4 * n * n]))
            assert err < 5e-3   # O(h^2) discretisation error of the manufactured solution
    assert its["mg"][0] < 100 and its["mg"][0] < its["cheb4"][0], its


def test_fgmres_captured_preconditioner_matches_eager():
    """fgmres replays a hipGraph of the preconditioner apply (capture_M, default): the residual history and the
    solution equal those with eager applies bit for bit (the apply is deterministic, the projections too)."""
    mp = _mp()
    n = 32
    _, (A, F, D, G), _ = _system(n)
    u, b = mp.manufactured_problem(n, etan=100.0, etas=1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("mg", 1), inner_P=mp.InnerSolver("mg", 1))
    out = {}
    for cap in (True, False):
        hist = []
        x, info = mp.fgmres(A, _cuda(b), M=pc, tol=1e-8, maxiter=60, residuals=hist, capture_M=cap)
        out[cap] = (x.cpu().numpy(), hist, info)
    assert out[True][2] == out[False][2] == 0
    assert out[True][1] == out[False][1]
    assert np.array_equal(_bits(out[True][0]), _bits(out[False][0]))
