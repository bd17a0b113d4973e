"""GPU parity of the segmented-reduction CSR SpMV (`mpbp_spmv_seg`, `DeviceCSR.matvec(order="seg")`).

Bar (BASELINE.json north_star): CSR indexing bit-exact, fp64 values within 1e-12 relative infinity norm of the
oracle (`oracle/csr_oracle.c`, the sequential row sums) -- the product is A @ u_vec (reference apply.py:72).
The kernel sums each row's entry pairs across lanes, so it is not bit-identical to the oracle; it is
deterministic (same bits run to run).
"""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import rel_inf

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

TOL = 1e-12   # north_star: relative infinity norm on fp64 results


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(oracle_built):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _mp():
    import mp_block_preconditioners_amd as mp
    return mp


def _cuda(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()


PARAMS = dict(xi=1.0, eta_n=100.0, eta_s=1.0, c=1.0, d_u=-1.0, d_p=1.0, d_div=-1.0)


@pytest.mark.parametrize("n", [3, 16, 100])
def test_seg_spmv_stencil_operators(n):
    """A (12 / 8 entries per row), F (10), D (8 per row: the 8-entry uniform path), G (2: the plain loop),
    every epilogue mode, against the oracle's sequential sums."""
    mp = _mp()
    from oracle import csr_oracle as co
    from oracle.stokes_oracle import StokesSystem
    osys = StokesSystem(n, products=False, **PARAMS)
    rng = np.random.default_rng(100 + n)
    for M in (osys.A, osys.F, osys.D, osys.G):
        dM = mp.DeviceCSR.from_scipy(M)
        x = rng.standard_normal(M.shape[1])
        z = rng.standard_normal(M.shape[0])
        for mode in (0, 1, 2):
            ref = co.spmv(M, x, z, mode=mode)
            got = dM.matvec(_cuda(x), mode=mode, z=_cuda(z), order="seg").cpu().numpy()
            assert rel_inf(got, ref) <= TOL, (M.shape, mode, rel_inf(got, ref))


@pytest.mark.parametrize("maxlen", [13, 200])
def test_seg_spmv_ragged_rows(maxlen):
    """Ragged and empty rows, odd wave starts, a uniform 64-row run, a partial last wave (the kernel's plain
    loop and its uniform path side by side)."""
    mp = _mp()
    from oracle import csr_oracle as co
    rng = np.random.default_rng(maxlen)
    lengths = rng.integers(0, maxlen + 1, size=3001)
    lengths[:70] = 0
    lengths[128:256] = 12
    rows = np.repeat(np.arange(lengths.size), lengths)
    M = sp.csr_matrix((rng.standard_normal(rows.size), (rows, rng.integers(0, 4000, size=rows.size))),
                      shape=(lengths.size, 4000))
    M.sum_duplicates()
    x, z = rng.standard_normal(4000), rng.standard_normal(lengths.size)
    dM = mp.DeviceCSR.from_scipy(M)
    for mode in (0, 1, 2):
        ref = co.spmv(M, x, z, mode=mode)
        got = dM.matvec(_cuda(x), mode=mode, z=_cuda(z), order="seg").cpu().numpy()
        assert rel_inf(got, ref) <= TOL, (mode, rel_inf(got, ref))
    assert np.all(dM.matvec(_cuda(x), order="seg").cpu().numpy()[:70] == 0.0)


def test_seg_spmv_1024_against_oracle():
    """configs[2]: the whole 1024^2 A (5.2 M rows, 58.7 M entries) -- the north_star measurement's operator --
    against the oracle's sequential sums over the same CSR arrays; deterministic run to run; the row sums of
    the sequential kernel stay bit-exact beside it."""
    mp = _mp()
    from oracle import csr_oracle as co
    bp = mp.MultiphaseBlockPreconditioner(1024, 1.0, 100.0, 1.0)
    A = bp.get_big_A_matrix(c=1.0, d_u=-1.0)[0]
    gen = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(A.shape[1], dtype=torch.float64, device="cuda", generator=gen)
    y1 = A.matvec(x, order="seg")
    y2 = A.matvec(x, order="seg")
    assert torch.equal(y1.view(torch.int64), y2.view(torch.int64)), "not deterministic"
    ys = A.matvec(x)
    ref = co.spmv(A.to_scipy(), x.cpu().numpy())
    assert np.array_equal(ys.cpu().numpy().view(np.uint64), ref.view(np.uint64))
    assert rel_inf(y1.cpu().numpy(), ref) <= TOL, rel_inf(y1.cpu().numpy(), ref)


@pytest.mark.parametrize("n", [3, 64])
def test_wave_table_same_bits(n):
    """The CSR SpMV started from the row blocks' wave table (default) == started from row_ptr (kernel option csr_table = 0) ==
    the oracle, bit for bit: stencil operators (uniform waves) and a ragged matrix (table flags 0), every mode."""
    mp = _mp()
    from oracle import csr_oracle as co
    from oracle.stokes_oracle import StokesSystem
    from mp_block_preconditioners_amd._lib import kernel_options
    osys = StokesSystem(n, products=False, **PARAMS)
    rng = np.random.default_rng(n)
    lengths = rng.integers(0, 30, size=2000)
    lengths[64:192] = 12
    rows = np.repeat(np.arange(lengths.size), lengths)
    R = sp.csr_matrix((rng.standard_normal(rows.size), (rows, rng.integers(0, 3000, size=rows.size))),
                      shape=(lengths.size, 3000))
    R.sum_duplicates()
    for M in (osys.A, osys.F, osys.D, R):
        dM = mp.DeviceCSR.from_scipy(M)
        assert dM.blocks.table is not None
        x, z = rng.standard_normal(M.shape[1]), rng.standard_normal(M.shape[0])
        for mode in (0, 1, 2):
            ref = co.spmv(M, x, z, mode=mode)
            for on in (1, 0):
                with kernel_options(csr_table=on):
                    got = dM.matvec(_cuda(x), mode=mode, z=_cuda(z)).cpu().numpy()
                assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), (M.shape, mode, on)


def test_row_blocks_of_another_matrix_refused():
    """the wave-table fast path trusts the row lengths of the row_ptr a plan was made from, so matvec refuses
    blocks planned for another matrix of the same shape."""
    import mp_block_preconditioners_amd as mp
    bp = mp.MultiphaseBlockPreconditioner(16, 1.0, 100.0, 1.0)
    A, _, F, _, _ = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    A2 = bp.get_big_A_matrix(c=1.0, d_u=-1.0)[0]
    x = torch.randn(A.shape[1], dtype=torch.float64, device="cuda")
    assert torch.equal(A.matvec(x, blocks=A.plan_blocks()), A.matvec(x))
    with pytest.raises(ValueError):
        A.matvec(x, blocks=A2.plan_blocks())
