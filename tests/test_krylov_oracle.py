"""The reproducible inner product's restatement (oracle/krylov_oracle.py, the checker of mpbp_rdot): its result depends
only on the set of terms -- any split of the vector, any order of the pieces, any grouping of the fold sums -- and it is
as accurate as the 3-fold analysis says.  (The GPU kernel is checked against it bit for bit in test_gpu_krylov.py.)"""
import math

import numpy as np
import pytest

from oracle.krylov_oracle import finish, fold_terms, gs_update, rd_sigmas, rdot, rdot_folds


@pytest.mark.parametrize("n,scale", [(1, 1.0), (1000, 1.0), (4097, 1e-200), (100003, 1e150), (5000, 1e-300)])
def test_rdot_is_order_and_split_independent(n, scale):
    rng = np.random.default_rng(n)
    w = rng.standard_normal(n) * scale
    V = rng.standard_normal((3, n)) * np.array([[1.0], [1e-8], [1e8]])
    V[1, ::7] = 0.0
    ref = rdot(V, w)
    bv, bw = np.max(np.abs(V), axis=1), float(np.max(np.abs(w)))
    for trial in range(4):
        perm = rng.permutation(n)
        cuts = np.sort(rng.choice(np.arange(1, n), size=min(5, max(n - 1, 0)), replace=False)) if n > 1 else []
        acc = np.zeros(9)
        for piece in np.split(perm, cuts):   # ranks of a partition: same global bounds and length
            acc = acc + rdot_folds(V[:, piece], w[piece], n, bv, bw)   # fold sums add exactly, in any order
        assert np.array_equal(finish(acc).view(np.uint64), ref.view(np.uint64)), trial
    exact = np.array([math.fsum(V[i] * w) for i in range(3)])
    err = np.abs(ref - exact)
    bound = bv * bw
    if scale >= 1e-250:   # (near the subnormal range the lower folds are skipped: split-independent, less accurate)
        assert np.all(err <= np.abs(exact) * 2.0 ** -52 + bound * 2.0 ** -48), (err, exact)


def test_rdot_zero_and_nonfinite():
    assert rdot(np.zeros((1, 10)), np.zeros(10))[0] == 0.0
    assert math.isnan(rdot(np.ones((1, 3)), np.array([1.0, np.nan, 2.0]))[0])
    s = rd_sigmas(1.0, 1 << 20)
    assert s[0] == math.ldexp(1.5, 1 + 22) and s[1] == math.ldexp(1.5, 1 + 44 - 53)
    assert rd_sigmas(1e-320, 10)[2] == 0.0          # a fold whose extractor would be subnormal is skipped
    q = fold_terms(np.array([0.1, -0.3]), rd_sigmas(0.3, 2))
    assert np.array_equal(q.sum(axis=0), np.array([0.1, -0.3]))   # 3 folds capture these terms exactly


def test_gs_update_adds_in_order():
    rng = np.random.default_rng(1)
    V, w, h = rng.standard_normal((5, 50)), rng.standard_normal(50), rng.standard_normal(5)
    a = np.zeros(50)
    for i in range(5):
        a = a + V[i] * h[i]
    assert np.array_equal(gs_update(V, 5, h, w), w - a)
