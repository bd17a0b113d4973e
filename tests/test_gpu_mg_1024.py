"""The solving configuration pinned against the oracle at the headline size: the Schur apply with one multigrid V-cycle
per inner inverse (mg:1 / mg:1; solve.py:257-277 with the multigrid the reference's comments name, solve.py:266, 274)
at 1024^2 -- BASELINE configs[2] (eta_n = 100) and configs[3] (eta_n / eta_s = 1e4).

* exact numerics: bit-identical to oracle/mg_oracle.py's V-cycles (Galerkin levels by the sequential C SpGEMM, smoothing
  and transfers by the C SpMV) inside oracle/schur_oracle.py's composition, on the oracle's own assembly of the
  operators (tests/test_oracle_golden.py pins that assembly against the reference's fixtures).  At 1024^2 the library
  picks level kernels it does not pick at 256^2 (stencil values on the 1 M-row level 1, grouped rows on the small
  levels); this is their oracle check at the size they run at.
* fast numerics (the bench's): against the same oracle output.  Bar: max(1e-12, 4 x floor), floor = the EXACT apply's
  own response to a one-ulp relative perturbation of its input (the exact GPU apply is the oracle's bits, checked in
  the first test).  No evaluation order other than the oracle's can sit closer to the oracle than that floor.  Measured
  (round 6, profiles/r06e_fast_tests_measured.txt): eta_n = 100 error 5.4e-12, floor 2.7e-12; eta ratio 1e4 error
  5.2e-12, floor 6.1e-12.  The measured error and floor are printed.
The oracle side costs about a minute of one host core per eta (assembly + products ~35 s, the F hierarchy ~25 s)."""
import numpy as np
import pytest

from conftest import rel_inf

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N = 1024
TOL_APPLY = 1e-12


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(oracle_built):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _cuda(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()


@pytest.fixture(scope="module", params=[100.0, 1.0e4], ids=["config2-eta100", "config3-eta1e4"])
def case(request):
    """(eta_n, oracle system, exact mg:1 / mg:1 preconditioner, its oracle hierarchies, input v, the oracle's apply)."""
    import mp_block_preconditioners_amd as mp
    from oracle import mg_oracle as mo
    from oracle.stokes_oracle import StokesSystem, theta_tables
    eta_n = request.param
    tabs = theta_tables(N)
    bp = mp.MultiphaseBlockPreconditioner(N, 1.0, eta_n, 1.0)
    bp.set_theta_tables(*tabs)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    kw = dict(inner_F=mp.InnerSolver("mg", 1), inner_P=mp.InnerSolver("mg", 1))
    exact = mp.ApproxSchurPreconditioner(F, D, G, **kw)
    S = StokesSystem(N, 1.0, eta_n, 1.0, 1.0, -1.0, tables=tabs)
    mF, mP = exact.mg_F, exact.mg_P
    oF = mo.MgOracle(S.F, mF.n, mF.fields, mF.pre, mF.post, mF.cycles, bounds=mF.bounds,
                     coarse_inv=mF.coarse_inv_host, coarsest=mF.coarsest)
    oP = mo.MgOracle(S.GtG, mP.n, mP.fields, mP.pre, mP.post, mP.cycles, bounds=mP.bounds,
                     coarse_inv=mP.coarse_inv_host, coarsest=mP.coarsest)
    assert [M.shape[0] for M, _ in oF.ops] == [M.shape[0] for M in mF.ops]
    v = np.random.default_rng(int(eta_n) + N).standard_normal(exact.shape[0])
    ref = _oracle_apply(S, oF, oP, v)
    yield dict(eta_n=eta_n, mp=mp, F=F, D=D, G=G, kw=kw, exact=exact, v=v, ref=ref)
    del exact
    torch.cuda.empty_cache()


def _oracle_apply(S, oF, oP, v):
    """approx_schur_op (solve.py:257-277) with the oracle V-cycles as both inner inverses (schur_oracle's order)."""
    from oracle import csr_oracle as co
    nu = S.F.shape[0]
    Finv_v = oF.solve(v[:nu])
    x_a = oP.solve(co.spmv(S.D, Finv_v, v[nu:], mode=1))
    x_p = oP.solve(co.spmv(S.GtFG, x_a))
    return np.concatenate([oF.solve(co.spmv(S.G, x_p), sub=Finv_v), x_p])


def test_1024_exact_mg_apply_bit_exact_vs_oracle(case):
    got = case["exact"].apply(_cuda(case["v"])).cpu().numpy()
    ref = case["ref"]
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), rel_inf(got, ref)
    # and its hipGraph replay (the bench's and the solver's launch mode)
    vt, out = _cuda(case["v"]), torch.zeros(ref.size, dtype=torch.float64, device="cuda")
    g = case["exact"].capture(vt, out)
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), ref.view(np.uint64))


def test_1024_fast_mg_apply_vs_oracle(case):
    mp = case["mp"]
    fast = mp.ApproxSchurPreconditioner(case["F"], case["D"], case["G"], case["exact"].GtG, case["exact"].GtFG,
                                        numerics="fast", **case["kw"])
    # the bench's solving configuration: level 1 of both hierarchies matrix-free in one launch, Gt_F_G's symmetric half
    assert fast.kernel_opts.mg_galerkin_mf == 2 and fast.kernel_opts.mg_galerkin_mf_p == 1
    assert fast.kernel_opts.q13_sym == 1
    v, ref = case["v"], case["ref"]
    got = fast.apply(_cuda(v)).cpu().numpy()
    sign = np.where(np.random.default_rng(3).random(v.size) < 0.5, -1.0, 1.0)
    v_ulp = v * (1.0 + sign * 2.0 ** -52)
    floor = rel_inf(case["exact"].apply(_cuda(v_ulp)).cpu().numpy(), ref)
    err = rel_inf(got, ref)
    print(f"eta_n={case['eta_n']:g}: fast vs oracle {err:.3e}, one-ulp floor {floor:.3e}")
    assert floor > 0.0
    assert 0.0 < err <= max(TOL_APPLY, 4.0 * floor), (err, floor)
