"""CPU checks of the multigrid stencil-values layout builder (mg.stencil_values_arrays, the host logic behind k_svl):
on the oracle's own Galerkin hierarchy, the layout's interior rows summed in slot order with columns row + delta
reproduce the oracle's sequential CSR sums bit for bit (the kernel's arithmetic, restated in numpy), and the edge
list is exactly the rows within `reach` of the periodic edge.  No GPU."""
import numpy as np
import pytest
import scipy.sparse as sp

torch = pytest.importorskip("torch")


def _hierarchy(n, which):
    from oracle.mg_oracle import hierarchy
    from oracle.stokes_oracle import StokesSystem
    from mp_block_preconditioners_amd.mg import FIELDS_PRESSURE, FIELDS_VELOCITY
    S = StokesSystem(n, xi=1.0, eta_n=100.0, eta_s=1.0, c=1.0, d_u=-1.0, d_p=1.0, d_div=-1.0, products=True)
    M, fields = (S.F, FIELDS_VELOCITY) if which == "F" else (S.GtG, FIELDS_PRESSURE)
    ops, _, _ = hierarchy(sp.csr_matrix(M), n, fields)
    return ops, len(fields)


@pytest.mark.parametrize("which", ["F", "GtG"])
def test_stencil_values_interior_sums_are_the_csr_sums(which, oracle_built):
    from oracle import csr_oracle as co
    from mp_block_preconditioners_amd.mg import stencil_values_arrays
    ops, nf = _hierarchy(32, which)
    rng = np.random.default_rng(3)
    checked = 0
    for A, m in ops[1:]:
        A = sp.csr_matrix(A)
        arr = stencil_values_arrays(torch.from_numpy(A.indptr.astype(np.int32)),
                                    torch.from_numpy(A.indices.astype(np.int32)), torch.from_numpy(A.data), nf, m)
        if arr is None:
            assert m < 16   # only the smallest levels may be too small for the stencil's reach
            continue
        R, K, delta, vals, edge = arr
        N = nf * m * m
        assert R % 2 == 0 and K == A.indptr[1] - A.indptr[0]
        delta, vals, edge = delta.numpy().reshape(nf, K), vals.numpy(), edge.numpy()
        x = rng.standard_normal(N)
        ref = co.spmv(A, x)
        rows = np.arange(N)
        f, cell = rows // (m * m), rows % (m * m)
        r, c = cell // m, cell % m
        interior = (r >= R) & (r < m - R) & (c >= R) & (c < m - R)
        assert np.array_equal(np.sort(edge), rows[~interior])
        ri = rows[interior]
        acc = np.zeros(ri.size)
        for s in range(K):   # the kernel's order: slot by slot, from 0.0
            acc = acc + vals[s * N + ri] * x[ri + delta[f[ri], s]]
        assert np.array_equal(acc.view(np.uint64), ref[ri].view(np.uint64))
        checked += 1
    assert checked >= 1


def test_stencil_values_refuses_other_operators():
    from mp_block_preconditioners_amd.mg import stencil_values_arrays
    rng = np.random.default_rng(0)
    A = sp.random(64, 64, density=0.1, format="csr", random_state=1)
    args = (torch.from_numpy(A.indptr.astype(np.int32)), torch.from_numpy(A.indices.astype(np.int32)),
            torch.from_numpy(A.data))
    assert stencil_values_arrays(*args, 1, 8) is None            # ragged rows
    n = 8
    I = sp.identity(n * n, format="csr") * rng.random()
    I.sort_indices()
    got = stencil_values_arrays(torch.from_numpy(I.indptr.astype(np.int32)), torch.from_numpy(I.indices.astype(np.int32)),
                                torch.from_numpy(I.data), 1, n)
    assert got is not None and got[0] == 0 and got[1] == 1 and got[4].numel() == 0   # a diagonal: no edge rows


def test_coarsest_level_size_is_capped():
    """a grid that coarsens to a large odd size (1000 -> 125) must refuse the dense coarsest inverse
    (4 * 125^2 = 62 500 rows: a 31 GB matrix and an O(m^3) pinv) with a clear error, before any allocation."""
    from types import SimpleNamespace
    from mp_block_preconditioners_amd import mg
    assert mg.level_sizes(1000, 16) == [1000, 500, 250, 125]
    with pytest.raises(ValueError, match="coarsest level has 62500 rows"):
        mg.dense_inverse_csr(SimpleNamespace(shape=(62500, 62500)))
