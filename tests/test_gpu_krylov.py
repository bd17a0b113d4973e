"""FGMRES's vector kernels on the GPU: the reproducible inner products (mpbp_rdot / mpbp_rdot_finish, mpbp_absmax)
bit for bit against oracle/krylov_oracle.py and independent of how the vector is split; and fgmres itself on the
reproducible kernels (the aliasing-safe work buffer, deterministic reruns)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lib():
    from mp_block_preconditioners_amd._lib import check, lib, ptr, stream_handle
    return check, lib, ptr, stream_handle


def _rdot(V, k, w, ntot, vb, wb):
    check, lib, ptr, sh = _lib()
    n = w.numel()
    part = torch.empty(max(1, int(lib().mpbp_rdot_part_size(n, k))), dtype=torch.float64, device="cuda")
    acc = torch.empty(3 * k, dtype=torch.float64, device="cuda")
    check(lib().mpbp_rdot(ptr(V), V.shape[1] if V.dim() == 2 else n, k, ptr(w), n, ntot, ptr(vb), ptr(wb), ptr(part),
                          ptr(acc), sh()))
    return acc


@pytest.mark.parametrize("k,n", [(1, 1), (3, 1000), (8, 4097), (37, 100003), (151, 5000), (5, 2_000_003)])
def test_rdot_matches_oracle_bit_for_bit(k, n):
    from oracle.krylov_oracle import finish, rdot_folds
    check, lib, ptr, sh = _lib()
    rng = np.random.default_rng(k * 7 + n)
    V = rng.standard_normal((k + 2, n)) * np.logspace(-6, 6, k + 2)[:, None]
    w = rng.standard_normal(n)
    vb, wb = np.max(np.abs(V[:k]), axis=1), float(np.max(np.abs(w)))
    dV, dw = torch.from_numpy(V).cuda(), torch.from_numpy(w).cuda()
    acc = _rdot(dV, k, dw, n, torch.from_numpy(vb).cuda(), torch.tensor([wb], dtype=torch.float64, device="cuda"))
    ref = rdot_folds(V[:k], w, n, vb, wb)
    assert np.array_equal(acc.cpu().numpy().view(np.uint64), ref.view(np.uint64))
    h = torch.empty(k, dtype=torch.float64, device="cuda")
    check(lib().mpbp_rdot_finish(k, ptr(acc), ptr(h), sh()))
    assert np.array_equal(h.cpu().numpy().view(np.uint64), finish(ref).view(np.uint64))
    # (against numpy's BLAS dot, itself off by ~sqrt(n) eps of the bound at n = 2e6)
    assert np.max(np.abs(h.cpu().numpy() - V[:k] @ w) / (vb * wb)) < 1e-12
    # absmax
    am = torch.empty(1, dtype=torch.float64, device="cuda")
    check(lib().mpbp_absmax(ptr(dw), n, ptr(am), sh()))
    assert float(am) == wb


def test_rdot_split_over_pieces_is_the_same():
    """Fold sums of a vector cut into pieces (the ranks of a row partition) add exactly: same bits as the whole."""
    rng = np.random.default_rng(4)
    n, k = 300_001, 6
    V = torch.from_numpy(rng.standard_normal((k, n))).cuda()
    w = torch.from_numpy(rng.standard_normal(n) * 1e3).cuda()
    vb = V.abs().amax(dim=1).contiguous()
    wb = w.abs().amax().reshape(1)
    whole = _rdot(V, k, w, n, vb, wb)
    acc = torch.zeros_like(whole)
    for a, b in ((0, 77_777), (77_777, 200_000), (200_000, n)):
        acc += _rdot(V[:, a:b].contiguous(), k, w[a:b].contiguous(), n, vb, wb)
    assert torch.equal(acc, whole)


@pytest.mark.parametrize("n,where", [(5_242_881, -1), (5_242_880, 0), (1_000_003, 777_777), (255, 254), (8 * 256 * 1024 + 5, -3)])
def test_absmax_large_vectors(n, where):
    """mpbp_absmax over FGMRES-sized vectors (unrolled grid-stride loads, per-workgroup atomics): the exact max |x|,
    wherever it sits (the unrolled body, the remainder loop, a negative entry)."""
    check, lib, ptr, sh = _lib()
    rng = np.random.default_rng(n)
    w = rng.standard_normal(n)
    w[where] = -1e3 * (1 + rng.random())
    dw = torch.from_numpy(w).cuda()
    am = torch.empty(1, dtype=torch.float64, device="cuda")
    check(lib().mpbp_absmax(ptr(dw), n, ptr(am), sh()))
    assert float(am) == float(np.max(np.abs(w)))


def test_rdot_nan_and_zero():
    check, lib, ptr, sh = _lib()
    w = torch.tensor([1.0, float("nan"), 2.0], dtype=torch.float64, device="cuda")
    am = torch.empty(1, dtype=torch.float64, device="cuda")
    check(lib().mpbp_absmax(ptr(w), 3, ptr(am), sh()))
    assert torch.isnan(am).all()
    acc = _rdot(w.reshape(1, 3).clone(), 1, w, 3, am, am)
    assert torch.isnan(acc).any()
    z = torch.zeros(10, dtype=torch.float64, device="cuda")
    acc = _rdot(z.reshape(1, 10).clone(), 1, z, 10, z[:1], z[:1])
    assert torch.equal(acc, torch.zeros(3, dtype=torch.float64, device="cuda"))


def test_fgmres_operator_return_value_not_modified():
    """a user operator that returns its input (identity) must not see fgmres's projections written into
    it; FGMRES on the identity converges in one iteration to x = b."""
    import mp_block_preconditioners_amd as mp
    b = torch.from_numpy(np.random.default_rng(2).standard_normal(1000)).cuda()
    seen = []

    def ident(x):
        seen.append(x)
        return x

    x, info = mp.fgmres(ident, b, tol=1e-12, maxiter=5)
    assert info == 0
    assert float((x - b).abs().max()) <= 1e-13 * float(b.abs().max())


def test_fgmres_is_deterministic():
    """Two solves of the same system give the same bits (reproducible reductions, captured preconditioner)."""
    import mp_block_preconditioners_amd as mp
    n = 32
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("mg", 1), inner_P=mp.InnerSolver("mg", 1))
    _, b = mp.manufactured_problem(n, 1.0, -1.0, 1.0, 100.0, 1.0)
    bd = torch.from_numpy(b).cuda()
    runs = []
    for _ in range(2):
        hist = []
        x, info = mp.fgmres(A, bd, M=pc, tol=1e-8, maxiter=60, residuals=hist)
        assert info == 0
        runs.append((x.clone(), list(hist)))
    assert torch.equal(runs[0][0], runs[1][0]) and runs[0][1] == runs[1][1]


@pytest.mark.parametrize("k,n", [(1, 1), (3, 1000), (8, 4097), (31, 70_001), (32, 4096), (33, 100_003), (40, 5000),
                                 (151, 20_000), (256, 3000), (12, 5_242_880)])
def test_gs_update_rdot_matches_oracle_bit_for_bit(k, n):
    """mpbp_gs_update_rdot (CGS2's first update and second projection in one pass) against
    oracle/krylov_oracle.py's gs_update_rdot: the updated vector bit-identical to mpbp_gs_update's, the fold sums to
    the restatement's under the a-priori bound -- with basis counts below, at and above the 32 kept in registers."""
    from oracle.krylov_oracle import finish, gs_update_rdot
    check, lib, ptr, sh = _lib()
    rng = np.random.default_rng(k * 11 + n)
    V = rng.standard_normal((k, n)) / np.sqrt(n)
    w = rng.standard_normal(n)
    h = V @ w
    vb = np.max(np.abs(V), axis=1) * (1.0 + 2.0 ** -50)
    wb = float(np.max(np.abs(w)))
    dV, dw = torch.from_numpy(V).cuda(), torch.from_numpy(w).cuda()
    dh, dvb = torch.from_numpy(h).cuda(), torch.from_numpy(vb).cuda()
    dwb = torch.tensor([wb], dtype=torch.float64, device="cuda")
    ref_w, ref_acc = gs_update_rdot(V, k, h, w, n, vb, wb)
    upd = torch.empty_like(dw)
    check(lib().mpbp_gs_update(ptr(dV), n, k, ptr(dh), ptr(dw), n, ptr(upd), sh()))
    part = torch.empty(max(1, int(lib().mpbp_rdot_part_size(n, k))), dtype=torch.float64, device="cuda")
    acc = torch.empty(3 * k, dtype=torch.float64, device="cuda")
    check(lib().mpbp_gs_update_rdot(ptr(dV), n, k, ptr(dh), ptr(dw), n, n, ptr(dvb), ptr(dwb), ptr(dw), ptr(part),
                                    ptr(acc), sh()))
    assert torch.equal(dw, upd)                                         # in place, mpbp_gs_update's bits
    assert np.array_equal(dw.cpu().numpy().view(np.uint64), ref_w.view(np.uint64))
    assert np.array_equal(acc.cpu().numpy().view(np.uint64), ref_acc.view(np.uint64))
    h2 = finish(ref_acc)
    assert np.max(np.abs(h2 - V @ ref_w)) <= 1e-12 * np.max(vb) * wb   # the second projection itself


def test_fgmres_fused_cgs2_matches_two_pass():
    """FGMRES with the fused CGS2 pass (fused_cgs2=True) and with the two projections apart: same convergence on the
    reference's problem (the second projection's bits differ only through its looser extractor bound)."""
    import mp_block_preconditioners_amd as mp
    n = 64
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("mg", 1), inner_P=mp.InnerSolver("mg", 1))
    _, b = mp.manufactured_problem(n, 1.0, -1.0, 1.0, 100.0, 1.0)
    bd = torch.from_numpy(b).cuda()
    out = {}
    for fused in (True, False):
        hist = []
        x, info = mp.fgmres(A, bd, M=pc, tol=1e-10, maxiter=100, residuals=hist, fused_cgs2=fused, ortho="cgs2")
        assert info == 0
        out[fused] = (x, hist)
    (x1, h1), (x2, h2) = out[True], out[False]
    assert abs(len(h1) - len(h2)) <= 1
    assert np.allclose(h1[: min(len(h1), len(h2))], h2[: min(len(h1), len(h2))], rtol=1e-6, atol=0)
    assert float((x1 - x2).abs().max()) <= 1e-8 * float(x2.abs().max())


@pytest.mark.parametrize("j,n", [(0, 1), (0, 1000), (1, 4097), (3, 100_003), (9, 5000), (31, 70_001), (40, 4096),
                                 (12, 5_242_880)])
def test_dcgs2_step_matches_oracle_bit_for_bit(j, n):
    """DCGS2's iteration j on the GPU -- mpbp_rdot2 (both columns' fold sums in one pass over V[0..j]) and
    mpbp_dcgs2_update (the scalars r, c, the bound, then V[j] <- q_j and V[j+1] <- u_{j+1}) -- against
    oracle/krylov_oracle.py's rdot2_folds / dcgs2_coeffs / dcgs2_update, bit for bit."""
    from oracle.krylov_oracle import dcgs2_coeffs, dcgs2_update, rdot2_folds
    check, lib, ptr, sh = _lib()
    rng = np.random.default_rng(j * 13 + n)
    Q, _ = np.linalg.qr(rng.standard_normal((n, j))) if 0 < j <= n else (np.zeros((n, 0)), None)
    V = np.zeros((j + 2, n))
    V[:j] = Q.T[:j]
    u = rng.standard_normal(n)
    u = u / np.linalg.norm(u) if j == 0 else u - 0.9 * (Q @ (Q.T @ u))   # j > 0: partly projected, not unit
    V[j] = u
    w = rng.standard_normal(n) * 3.0
    vb = np.ones(j + 2)
    vb[j] = 1.0 if j == 0 else float(np.max(np.abs(u))) * (1 + 2.0 ** -40)
    wb = float(np.max(np.abs(w)))
    dV, dw = torch.from_numpy(V.copy()).cuda(), torch.from_numpy(w).cuda()
    dvb = torch.from_numpy(vb).cuda()
    dwb = torch.tensor([wb], dtype=torch.float64, device="cuda")
    part = torch.empty(max(1, int(lib().mpbp_rdot_part_size(n, 2 * (j + 1)))), dtype=torch.float64, device="cuda")
    acc = torch.empty(6 * (j + 1), dtype=torch.float64, device="cuda")
    check(lib().mpbp_rdot2(ptr(dV), n, j + 1, ptr(dV[j]), ptr(dw), n, n, ptr(dvb), ptr(dvb[j:j + 1]), ptr(dwb),
                           ptr(part), ptr(acc), sh()))
    ref_acc = rdot2_folds(V[: j + 1], V[j], w, n, vb[: j + 1], vb[j], wb)
    assert np.array_equal(acc.cpu().numpy().view(np.uint64), ref_acc.view(np.uint64))
    hu = torch.empty(256, dtype=torch.float64, device="cuda")
    hw = torch.empty(256, dtype=torch.float64, device="cuda")
    P = torch.empty(4, dtype=torch.float64, device="cuda")
    check(lib().mpbp_dcgs2_update(ptr(dV), n, j, ptr(acc), ptr(dwb), ptr(dw), n, 1, ptr(hu), ptr(hw), ptr(P), sh()))
    rhu, rhw, rP = dcgs2_coeffs(j, ref_acc, wb)
    dcgs2_update(V, j, rhu, rhw, rP, w)
    assert np.array_equal(hu[: j + 1].cpu().numpy().view(np.uint64), rhu.view(np.uint64))
    assert np.array_equal(hw[: j + 1].cpu().numpy().view(np.uint64), rhw.view(np.uint64))
    assert np.array_equal(P.cpu().numpy().view(np.uint64), rP.view(np.uint64))
    assert np.array_equal(dV.cpu().numpy().view(np.uint64), V.view(np.uint64))
    # what the step means: q_j unit and orthogonal to V[0..j-1]; u_{j+1} orthogonal to V[0..j] (one CGS pass); the bound
    assert abs(np.linalg.norm(V[j]) - 1.0) < 1e-12
    if j:
        assert np.max(np.abs(V[:j] @ V[j])) < 1e-12
    assert np.max(np.abs(V[: j + 1] @ V[j + 1])) < 1e-10 * np.linalg.norm(w)
    assert np.max(np.abs(V[j + 1])) <= rP[3]


@pytest.mark.parametrize("n,inner", [(64, "mg:1"), (256, "mg:1"), (256, "chebyshev:4")])
def test_fgmres_dcgs2_matches_cgs2(n, inner):
    """FGMRES with DCGS2 (the default: two basis passes per iteration) and with CGS2 (four): the reference's
    manufactured problem (solve.py:52-80) converges in the same iterations (within 2), to the same solution within the
    tolerance, and each is deterministic."""
    import mp_block_preconditioners_amd as mp
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    kind, k = inner.split(":")
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver(kind, int(k)), inner_P=mp.InnerSolver(kind, int(k)),
                                      numerics="fast")
    _, b = mp.manufactured_problem(n, 1.0, -1.0, 1.0, 100.0, 1.0)
    bd = torch.from_numpy(b).cuda()
    out = {}
    for ortho in ("dcgs2", "cgs2", "dcgs2"):
        hist = []
        x, info = mp.fgmres(A, bd, M=pc, tol=1e-8, maxiter=150, residuals=hist, ortho=ortho)
        if ortho in out:
            assert torch.equal(x, out[ortho][0]) and hist == out[ortho][1]   # deterministic
        out[ortho] = (x, hist, info)
    (xd, hd, id_), (xc, hc, ic) = out["dcgs2"], out["cgs2"]
    assert id_ == ic
    if ic == 0:
        assert abs(len(hd) - len(hc)) <= 2, (len(hd), len(hc))
        true = float(torch.linalg.vector_norm(bd - A.matvec(xd)))
        assert true <= 1.01e-8 * hd[0]
        assert float((xd - xc).abs().max()) <= 1e-6 * float(xc.abs().max())
    else:   # chebyshev:4 stalls: both reach maxiter without converging.  Once the Krylov space
        # stops growing, DCGS2's r = sqrt(alpha - s.s) cancels to 0 (u_j within ~1e-7 of span(V)): the cycle ends
        # there and restarts from the true residual, where CGS2 goes on normalising rounding noise
        assert ic == id_ == 150 and len(hc) == 151 and len(hd) == 151
        assert min(hd) > 0.0 and min(hc) > 0.0   # a cancelled r_j records the restart's true residual, not a false 0
        for x in (xd, xc):
            true = float(torch.linalg.vector_norm(bd - A.matvec(x)))
            assert true <= hd[0]
