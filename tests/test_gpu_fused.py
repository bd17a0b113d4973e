"""Fused launches of the apply against the per-sweep launches they replace, bit for bit.

k_gtg_solve runs a whole Chebyshev Gt_G solve (solve.py:265 / 271) as one tiled launch: level 0 (x0 = c2 b / diag)
and every sweep recomputed over a shrinking halo in LDS, each row and update with the per-sweep kernels' IEEE
operations -- so the apply must not change by a bit whether it is on (default) or off, in both F numerics, on grids
smaller than, equal to and not a multiple of the 64 x 8 tile.  The exact apply with it on is also pinned against the
oracle by tests/test_gpu_configs.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(oracle_built):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("n", [3, 5, 17, 64, 82, 100, 128, 256, 300])
@pytest.mark.parametrize("kp", [2, 3, 4, 6])
@pytest.mark.parametrize("numerics", ["exact", "fast"])
def test_fused_gtg_solve_equals_per_sweep(n, kp, numerics):
    import mp_block_preconditioners_amd as mp
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("chebyshev", 4),
                                      inner_P=mp.InnerSolver("chebyshev", kp), numerics=numerics)
    assert pc.pg_stencil is not None
    v = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda",
                    generator=torch.Generator(device="cuda").manual_seed(n * 10 + kp))
    pc.set_kernel_opts(gtg_fused=0)
    ref = pc.apply(v).clone()
    pc.set_kernel_opts(gtg_fused=1)
    got = pc.apply(v)
    assert torch.equal(got, ref), float((got - ref).abs().max())


def test_fused_gtg_solve_vs_oracle_256():
    """configs[1] with the fused pressure solves: the whole apply bit-exact against oracle/schur_oracle.py."""
    import mp_block_preconditioners_amd as mp
    from oracle.schur_oracle import Inner, approx_schur_apply
    from oracle.stokes_oracle import StokesSystem, theta_tables
    n = 256
    tabs = theta_tables(n)
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    bp.set_theta_tables(*tabs)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("chebyshev", 4),
                                      inner_P=mp.InnerSolver("chebyshev", 5))
    osys = StokesSystem(n, 1.0, 100.0, 1.0, 1.0, -1.0, tables=tabs)
    v = np.random.default_rng(7).standard_normal(pc.shape[0])
    got = pc.apply(torch.from_numpy(v).cuda()).cpu().numpy()
    ref = approx_schur_apply(osys.F, osys.D, osys.G, osys.GtG, osys.GtFG, v,
                             Inner("chebyshev", 4, pc.inner_F.lmin, pc.inner_F.lmax),
                             Inner("chebyshev", 5, pc.inner_P.lmin, pc.inner_P.lmax))
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("n", [3, 5, 17, 64, 76, 100, 128, 255, 256, 300])
@pytest.mark.parametrize("kf", [2, 3, 4, 5])
@pytest.mark.parametrize("fuse_g", [True, False])
def test_ftile_equals_marching(n, kf, fuse_g):
    """k_ftile (x0 + the first sweep, and the last pair, of a fast F solve on 2D tiles) performs the marching kernels'
    tolerance-mode operations: the apply is bit-identical with the tiles on and off (marching k_march_init, k_march,
    k_march2), with G x_p recomputed in the second solve and launched separately."""
    import mp_block_preconditioners_amd as mp
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("chebyshev", kf),
                                      inner_P=mp.InnerSolver("chebyshev", 4), numerics="fast", fuse_g=fuse_g)
    v = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda",
                    generator=torch.Generator(device="cuda").manual_seed(n * 10 + kf))
    pc.set_kernel_opts(f_solve=0, f_tile=0)   # (the whole-solve launch would take over kf = 3, 4 either way)
    ref = pc.apply(v).clone()
    pc.set_kernel_opts(f_tile=1)
    got = pc.apply(v)
    assert torch.equal(got, ref), float((got - ref).abs().max())


@pytest.mark.parametrize("n", [3, 5, 64, 70, 71, 72, 76, 100, 128, 255, 256, 300])
@pytest.mark.parametrize("kf", [2, 3, 4, 5])
@pytest.mark.parametrize("fuse_g", [True, False])
@pytest.mark.parametrize("tile", [0, 1], ids=["64x8", "32x16"])
def test_fsolve_equals_ftile(n, kf, fuse_g, tile):
    """k_fsolve (a whole fast F solve of 3 or 4 updates in one tiled launch: x0 and every sweep over a shrinking halo,
    each cell's state in its owning lane) performs the k_ftile launches' operations: the apply is bit-identical with it
    on and off, with G x_p recomputed in the second solve and launched separately, on grids below, at and above its
    minimum (n >= 70 for 3 updates, 72 for 4) and not multiples of the 64 x 8 tile -- in each tile form (kernel option
    f_solve_tile: the 64 x 8 tile, and the 32 x 16 tile with the rings spread over the waves and cached row terms)."""
    import mp_block_preconditioners_amd as mp
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("chebyshev", kf),
                                      inner_P=mp.InnerSolver("chebyshev", 4), numerics="fast", fuse_g=fuse_g)
    v = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda",
                    generator=torch.Generator(device="cuda").manual_seed(n * 10 + kf + 7))
    pc.set_kernel_opts(f_solve=0)
    ref = pc.apply(v).clone()
    pc.set_kernel_opts(f_solve=1, f_solve_tile=tile)
    got = pc.apply(v)
    assert torch.equal(got, ref), float((got - ref).abs().max())


@pytest.mark.parametrize("n", [128, 256])
def test_ftile_multigrid_smoothing_equals_marching(n):
    """Multigrid level 0 with fast F numerics: the pre-smoothing (x0 + one sweep) and the post-smoothing restart (two
    sweeps from d = 0, read as +0.0 instead of a memset) on tiles are bit-identical to the marching sweeps."""
    import mp_block_preconditioners_amd as mp
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("mg", 1), inner_P=mp.InnerSolver("mg", 1),
                                      numerics="fast")
    v = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda",
                    generator=torch.Generator(device="cuda").manual_seed(n))
    pc.set_kernel_opts(f_tile=0)
    ref = pc.apply(v).clone()
    pc.set_kernel_opts(f_tile=1)
    got = pc.apply(v)
    assert torch.equal(got, ref), float((got - ref).abs().max())


@pytest.mark.parametrize("n", [5, 17, 64, 128])
@pytest.mark.parametrize("kf", [3, 5])
def test_fdirect_equals_marching(n, kf):
    """Kernel option f_direct = 1: the per-sweep tolerance-mode F launches on the direct kernel (one thread per cell) perform
    the marching kernels' rows4 operations -- the apply is bit-identical (whole-solve and tile launches off)."""
    import mp_block_preconditioners_amd as mp
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("chebyshev", kf),
                                      inner_P=mp.InnerSolver("chebyshev", 4), numerics="fast")
    v = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda",
                    generator=torch.Generator(device="cuda").manual_seed(n * 10 + kf + 3))
    pc.set_kernel_opts(f_solve=0, f_tile=0, f_pair=0)
    ref = pc.apply(v).clone()
    pc.set_kernel_opts(f_direct=1)
    got = pc.apply(v)
    assert torch.equal(got, ref), float((got - ref).abs().max())


@pytest.mark.parametrize("n", [82, 100, 128, 256])
@pytest.mark.parametrize("numerics", ["exact", "fast"])
def test_gtg_solve_builds_rhs_equals_d_launch(n, numerics):
    """The first fused Gt_G solve building rhs = D Finv_v + v_p per staged cell (DStencilDev::row's operations, EpiAdd's
    sum) is bit-identical to the D launch writing rhs, in both numerics, with 256- and 512-lane workgroups."""
    import mp_block_preconditioners_amd as mp
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("chebyshev", 4),
                                      inner_P=mp.InnerSolver("chebyshev", 4), numerics=numerics)
    v = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda",
                    generator=torch.Generator(device="cuda").manual_seed(n + 5))
    pc.set_kernel_opts(gtg_drhs=0)
    ref = pc.apply(v).clone()
    pc.set_kernel_opts(gtg_drhs=1)
    got = pc.apply(v).clone()
    pc.set_kernel_opts(gtg_tpb=256)
    got256 = pc.apply(v).clone()
    assert torch.equal(got, ref), float((got - ref).abs().max())
    assert torch.equal(got256, ref), float((got256 - ref).abs().max())
