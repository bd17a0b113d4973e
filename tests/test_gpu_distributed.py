"""The row-partitioned GPU apply (DistributedSchurPreconditioner: halo callbacks inside
mpbp_schur_apply, interior/boundary SELL slices) on one GPU with two gloo ranks, bit for bit
against the single-GPU apply of the global system.  (RCCL needs one GPU per rank; the driver's
multi-GPU bench exercises the same code over RCCL.)"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, layout, f_mode, kind, errfile, ca="auto", fuse_g=True, numerics="exact"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import mp_block_preconditioners_amd as mpb
        from mp_block_preconditioners_amd.distributed import DistributedSchurPreconditioner
        iF, iP = mpb.InnerSolver("chebyshev", 4), mpb.InnerSolver("chebyshev", 3)
        dpc = DistributedSchurPreconditioner(n, 1.0, 100.0, 1.0, inner_F=iF, inner_P=iP, layout=layout,
                                             f_mode=f_mode, ca=ca, fuse_g=fuse_g, numerics=numerics,
                                             kernel_opts={"march_rows": kind})
        assert dpc.fuse_g == bool(fuse_g and dpc.ca)
        assert (dpc.f_stencil is not None) == (f_mode != "assembled")
        if ca is True:
            assert dpc.ca and dpc.h_u == dpc.ca_q + 2 + 1 + 3, (dpc.h_u, dpc.ca_q)
        if numerics == "fast" and n >= 5:   # Gt_F_G's symmetric half over the rank's row block (k_q13p), as one GPU
            assert dpc.q13 is not None and dpc.kernel_opts.q13_sym == 1
        bp = mpb.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
        _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
        # the reference: the assembled one-GPU apply (exact numerics), or the one-GPU apply with the same fast rows
        # (the partition reads Gt_F_G's symmetric half over its row block, as the one-GPU default does)
        pc = mpb.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP, layout=layout,
                                           f_mode="assembled" if numerics == "exact" else "stencil", numerics=numerics,
                                           kernel_opts={"q13_mf": 0})
        assert (pc.inner_F.lmin, pc.inner_F.lmax) == (dpc.inner_F.lmin, dpc.inner_F.lmax)
        v = torch.from_numpy(np.random.default_rng(5).standard_normal(pc.shape[0])).cuda()
        gids = torch.from_numpy(dpc.local_to_global_rows()).cuda()
        ref = pc.apply(v)[gids]
        for _ in range(2):
            # (the per-sweep schedule's fast F solves start from x0 = (c2 b) (1 / diag) with the fast reciprocal
            # diagonals, k_f_fast_init, as the one-GPU fast first sweep: the same bits in both numerics)
            got = dpc.apply(v[gids].contiguous())
            assert torch.equal(got, ref), float((got - ref).abs().max())
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise


@pytest.mark.parametrize("world,n,layout,f_mode,kind", [(2, 64, "sell", "stencil", 4), (2, 64, "sell", "assembled", 4),
                                                        (2, 64, "csr", "assembled", 2), (3, 50, "sell", "stencil", 1),
                                                        (4, 9, "csr", "stencil", 1), (2, 64, "sell", "stencil", 3),
                                                        (3, 50, "sell", "stencil", 6), (4, 9, "sell", "stencil", 3),
                                                        (2, 64, "sell", "stencil", 0), (3, 50, "csr", "stencil", 0)])
def test_distributed_apply_matches_single_gpu(world, n, layout, f_mode, kind, tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    errfile = str(tmp_path / "err.txt")
    try:
        mp.spawn(_worker, args=(world, _free_port(), n, layout, f_mode, kind, errfile), nprocs=world, join=True)
    except Exception:
        msg = open(errfile).read() if os.path.exists(errfile) else ""
        pytest.fail(f"distributed worker failed:\n{msg}")


@pytest.mark.parametrize("world,n,layout,ca,fuse_g", [(2, 64, "sell", True, True), (2, 64, "sell", False, True),
                                                     (3, 50, "csr", True, True), (4, 40, "sell", True, True),
                                                     (2, 64, "sell", True, False), (3, 50, "sell", True, False)])
def test_distributed_apply_ca_schedule(world, n, layout, ca, fuse_g, tmp_path):
    """The communication-avoiding schedule (2 exchanges per apply, ghost rows recomputed; the second F solve with
    G x_p recomputed from x_p's ghost rows, and with the G launch) and the per-sweep one, 2-4 gloo ranks on one
    GPU, bit for bit against the single-GPU apply."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    errfile = str(tmp_path / "err.txt")
    try:
        mp.spawn(_worker, args=(world, _free_port(), n, layout, "stencil", 4, errfile, ca, fuse_g), nprocs=world,
                 join=True)
    except Exception:
        msg = open(errfile).read() if os.path.exists(errfile) else ""
        pytest.fail(f"distributed worker failed:\n{msg}")


@pytest.mark.parametrize("world,n,ca", [(2, 64, True), (3, 50, True), (2, 64, False)])
def test_distributed_fast_numerics_matches_single_gpu(world, n, ca, tmp_path):
    """Tolerance-mode F numerics under the row partition: the CA schedule (the default) and the per-sweep schedule (its
    F solves starting from the fast reciprocal diagonals, k_f_fast_init) run the same fast rows and updates per grid
    point as one GPU -- bit for bit."""
    errfile = str(tmp_path / "err.txt")
    _spawn(_worker, (world, _free_port(), n, "sell", "stencil", 4, errfile, ca, True, "fast"), world, errfile)


def _self_halo_worker(_index, port, n, halo, f_mode, pg_mode, kind, graph, errfile, overlap=False, ca="auto",
                      inner=(("chebyshev", 4), ("chebyshev", 3))):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=0, world_size=1)
        import mp_block_preconditioners_amd as mpb
        from mp_block_preconditioners_amd.distributed import DistributedSchurPreconditioner
        iF, iP = mpb.InnerSolver(*inner[0]), mpb.InnerSolver(*inner[1])
        dpc = DistributedSchurPreconditioner(n, 1.0, 100.0, 1.0, inner_F=iF, inner_P=iP, f_mode=f_mode,
                                             pg_mode=pg_mode, halo=halo, self_halo=True, halo_overlap=overlap,
                                             ca=ca, kernel_opts={"march_rows": kind})
        if ca is True:
            assert dpc.ca
        assert dpc.partitioned and dpc.nu_ext > dpc.nu
        bp = mpb.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
        _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
        pc = mpb.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP, f_mode="assembled", pg_mode="assembled")
        v = torch.from_numpy(np.random.default_rng(9).standard_normal(pc.shape[0])).cuda()
        ref = pc.apply(v)
        for _ in range(2):
            got = dpc.apply(v.clone())
            assert torch.equal(got, ref), float((got - ref).abs().max())
        if graph:   # in-order RCCL halo: captured (thread-local error mode); other halos are refused
            vin, out = v.clone(), torch.zeros_like(v)
            if halo == "rccl" and not overlap:
                g = dpc.capture(vin, out)
                out.zero_()
                g.replay()
                torch.cuda.synchronize()
                assert torch.equal(out, ref)
                vin.copy_(2.0 * v)
                g.replay()
                assert torch.equal(out, pc.apply(2.0 * v))
                del g
            else:
                try:
                    dpc.capture(vin, out)
                    raise AssertionError("capture of this partitioned apply should be refused")
                except NotImplementedError:
                    pass
        dpc.close()
        dist.destroy_process_group()
    except BaseException as e:
        with open(errfile, "a") as f:
            f.write(f"{type(e).__name__}: {e}\n")
        raise


@pytest.mark.parametrize("n,halo,f_mode,pg_mode,kind,graph,overlap", [
    (64, "rccl", "stencil", "stencil", 4, False, False), (50, "rccl", "assembled", "assembled", 4, False, False),
    (33, "rccl", "stencil", "assembled", 1, False, False), (64, "torch", "stencil", "stencil", 4, False, False),
    (64, "rccl", "stencil", "stencil", 4, True, False), (64, "rccl", "stencil", "stencil", 4, False, True),
    (64, "torch", "stencil", "stencil", 4, True, False),
    (40, "rccl", "assembled", "stencil", 4, False, True)])
def test_self_halo_partitioned_apply(n, halo, f_mode, pg_mode, kind, graph, overlap, tmp_path, ca="auto",
                                     inner=(("chebyshev", 4), ("chebyshev", 3))):
    """One rank runs the partitioned apply with ghost rows filled by the periodic self-exchange -- the
    RCCL point-to-point halo (libmpbp's own communicator) and the torch one -- bit for bit against the
    single-GPU apply."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    errfile = str(tmp_path / "err.txt")
    try:
        mp.spawn(_self_halo_worker, args=(_free_port(), n, halo, f_mode, pg_mode, kind, graph, errfile, overlap, ca,
                                          inner),
                 nprocs=1, join=True)
    except Exception:
        msg = open(errfile).read() if os.path.exists(errfile) else ""
        pytest.fail(f"self-halo worker failed:\n{msg}")


@pytest.mark.parametrize("halo,ca", [("rccl", False), ("rccl", True), ("torch", True)])
def test_self_halo_ca_schedule(halo, ca, tmp_path):
    """RCCL / torch self-exchange with and without the communication-avoiding schedule."""
    test_self_halo_partitioned_apply(48, halo, "stencil", "stencil", 4, False, False, tmp_path, ca=ca)


@pytest.mark.parametrize("inner", [(("jacobi", 1), ("jacobi", 1)), (("jacobi", 2), ("chebyshev", 2)),
                                   (("chebyshev", 6), ("jacobi", 3)), (("chebyshev", 3), ("chebyshev", 5))],
                         ids=["jac1-jac1", "jac2-cheb2", "cheb6-jac3", "cheb3-cheb5"])
def test_self_halo_ca_inner_solvers(inner, tmp_path):
    """The CA schedule's ghost-row depths for other inner solvers: one-sweep (init only) solves, Jacobi,
    deeper Chebyshev -- bit for bit against the single-GPU apply (RCCL self-exchange)."""
    test_self_halo_partitioned_apply(40, "rccl", "stencil", "stencil", 4, False, False, tmp_path, ca=True,
                                     inner=inner)


def _rccl_worker(rank, world, port, n, ca, errfile):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(rank)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
        import mp_block_preconditioners_amd as mpb
        from mp_block_preconditioners_amd.distributed import DistributedSchurPreconditioner
        iF, iP = mpb.InnerSolver("chebyshev", 4), mpb.InnerSolver("chebyshev", 4)
        dpc = DistributedSchurPreconditioner(n, 1.0, 100.0, 1.0, inner_F=iF, inner_P=iP, halo="rccl", ca=ca,
                                             device=f"cuda:{rank}")
        bp = mpb.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0, device=f"cuda:{rank}")
        _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
        pc = mpb.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP)
        v = torch.from_numpy(np.random.default_rng(11).standard_normal(pc.shape[0])).to(f"cuda:{rank}")
        gids = torch.from_numpy(dpc.local_to_global_rows()).to(f"cuda:{rank}")
        ref = pc.apply(v)[gids]
        for _ in range(2):
            got = dpc.apply(v[gids].contiguous())
            assert torch.equal(got, ref), float((got - ref).abs().max())
        dist.barrier()
        dpc.close()
        dist.destroy_process_group()
    except BaseException as e:
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise


@pytest.mark.parametrize("world,n,ca", [(2, 256, True), (2, 256, False), (2, 130, True)])
def test_rccl_two_gpus_matches_single_gpu(world, n, ca, tmp_path):
    """The partitioned apply over RCCL point-to-point between two GPUs (one rank per GPU, libmpbp's own
    communicator), bit for bit against the single-GPU apply of the global system.  Runs where the node has
    two GPUs (the driver's multi-GPU box); skipped on a one-GPU box."""
    if not torch.cuda.is_available() or torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs")
    errfile = str(tmp_path / "err.txt")
    try:
        mp.spawn(_rccl_worker, args=(world, _free_port(), n, ca, errfile), nprocs=world, join=True)
    except Exception:
        msg = open(errfile).read() if os.path.exists(errfile) else ""
        pytest.fail(f"RCCL worker failed:\n{msg}")


# ---------------------------------------------------------------------------------------------------------------
# Row 17: the partitioned operator A u (DistributedMatrix) and FGMRES over the ranks; row 18: multigrid inner solves
# under the row partition (PartitionedMultigrid).  gloo ranks share the one GPU (RCCL needs a GPU per rank); the RCCL
# halo kinds are exercised by the self-exchange.

def _spawn(fn, args, nprocs, errfile):
    try:
        mp.spawn(fn, args=args, nprocs=nprocs, join=True)
    except Exception:
        msg = open(errfile).read() if os.path.exists(errfile) else ""
        pytest.fail(f"worker failed:\n{msg}")


def _matrix_worker(rank, world, port, n, overlap, halo, errfile):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import mp_block_preconditioners_amd as mpb
        from mp_block_preconditioners_amd.distributed import DistributedMatrix
        bp = mpb.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
        A = bp.get_big_A_matrix(c=1.0, d_u=-1.0)[0]
        dA = DistributedMatrix(A, n, 5, halo=halo, overlap=overlap, self_halo=(world == 1))
        assert dA.partitioned and dA.h == 1
        u = torch.from_numpy(np.random.default_rng(3).standard_normal(A.shape[0])).cuda()
        gids = torch.from_numpy(dA.local_to_global_rows()).cuda()
        ref = A.matvec(u)[gids]
        for _ in range(3):
            got = dA.apply(u[gids].contiguous())
            assert torch.equal(got, ref), float((got - ref).abs().max())
        dA.close()
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise


@pytest.mark.parametrize("world,n,overlap,halo", [(2, 64, False, "auto"), (3, 50, False, "auto"), (4, 9, False, "auto"),
                                                  (1, 64, False, "rccl"), (1, 64, True, "rccl"), (1, 33, True, "rccl"),
                                                  (1, 40, False, "torch")])
def test_distributed_matrix_matches_global_spmv(world, n, overlap, halo, tmp_path):
    """A u over the row partition (apply.py:72 on the 5-field system): the interior rows' SpMV, the ghost exchange
    (gloo ranks; the RCCL self-exchange in order and overlapped on the halo's side stream), the boundary rows --
    bit-identical to the rows of the one-GPU SpMV."""
    errfile = str(tmp_path / "err.txt")
    _spawn(_matrix_worker, (world, _free_port(), n, overlap, halo, errfile), world, errfile)


def _inner_pair(spec):
    import mp_block_preconditioners_amd as mpb
    (kf, sf), (kp, sp) = spec
    return mpb.InnerSolver(kf, sf), mpb.InnerSolver(kp, sp)


def _mg_worker(rank, world, port, n, inner, min_cells, halo, errfile, numerics="exact"):
    """The partitioned Schur apply with multigrid inner solves vs the one-GPU apply with its default kernel choices
    (fast numerics at n >= 72: level 1 matrix-free in one launch on both sides -- k_gal1 / k_gal1p over the rank's owned
    coarse rows under the partition)."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import mp_block_preconditioners_amd as mpb
        from mp_block_preconditioners_amd.distributed import (DistributedSchurPreconditioner, LocalHierarchy,
                                                              PartitionedMultigrid)
        iF, iP = _inner_pair(inner)
        dpc = DistributedSchurPreconditioner(n, 1.0, 100.0, 1.0, inner_F=iF, inner_P=iP, halo=halo,
                                             self_halo=(world == 1), mg_min_cells=min_cells, numerics=numerics)
        for m in (dpc.mg_F, dpc.mg_P):
            if m is not None:
                assert isinstance(m, PartitionedMultigrid) and 1 <= m.part_levels <= m.g.nlevels - 1
                if min_cells == 0 and world > 1:   # every level but the coarsest partitioned (where rows allow)
                    assert m.part_levels >= min(2, m.g.nlevels - 1), (m.part_levels, m.g.sizes)
                if world > 1:   # rank-local levels: this rank's band of rows, no global operator
                    assert isinstance(m.g, LocalHierarchy)
                    if min_cells:
                        assert m.g.band[0].shape[0] < m.nf * m.g.sizes[0] ** 2, (m.g.band[0].shape, m.g.sizes)
        bp = mpb.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
        _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
        pc = mpb.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP, numerics=numerics)
        v = torch.from_numpy(np.random.default_rng(8).standard_normal(pc.shape[0])).cuda()
        gids = torch.from_numpy(dpc.local_to_global_rows()).cuda()
        ref = pc.apply(v)[gids]
        for _ in range(2):
            got = dpc.apply(v[gids].contiguous())
            assert torch.equal(got, ref), float((got - ref).abs().max())
        if numerics == "fast" and n >= 72:   # the matrix-free level 1 ran: the stored one gives other bits
            dpc.kernel_opts.mg_galerkin_mf = 0
            stored = dpc.apply(v[gids].contiguous())
            assert not torch.equal(stored, ref)
            assert float((stored - ref).abs().max()) <= 1e-10 * float(ref.abs().max())
            dpc.kernel_opts.mg_galerkin_mf = 2
        if halo == "rccl":   # in-order RCCL halo: the partitioned MG apply captured into a hipGraph
            vin, out = v[gids].contiguous(), torch.zeros_like(ref)
            g = dpc.capture(vin, out)
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(out, ref)
            del g
        dpc.close()
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise


MG1 = (("mg", 1), ("mg", 1))


@pytest.mark.parametrize("world,n,inner,min_cells,halo", [
    (2, 64, MG1, 1 << 14, "auto"), (2, 64, MG1, 0, "auto"), (4, 64, MG1, 0, "auto"), (3, 48, MG1, 0, "auto"),
    (3, 50, MG1, 0, "auto"), (2, 64, (("mg", 2), ("chebyshev", 4)), 0, "auto"),
    (2, 64, (("chebyshev", 4), ("mg", 1)), 0, "auto"), (1, 64, MG1, 0, "rccl"), (1, 32, MG1, 0, "torch"),
    (2, 128, MG1, 0, "auto"), (4, 128, MG1, 0, "auto"), (3, 100, MG1, 0, "auto"), (2, 128, MG1, 1 << 14, "auto"),
    (1, 128, MG1, 0, "rccl")])
@pytest.mark.parametrize("numerics", ["exact", "fast"])
def test_partitioned_multigrid_apply_matches_single_gpu(world, n, inner, min_cells, halo, numerics, tmp_path):
    """Row 18: multigrid inner solves under the row partition -- level 0 the apply's own matrix-free F / Gt_G, the
    Galerkin levels row-partitioned down to part_levels (ghost rows per operator), the coarser levels all-gathered and
    replicated -- bit for bit against the one-GPU apply (2-4 gloo ranks; ceil-halved partitions at n = 50; the RCCL
    self-exchange, captured).  With 2+ ranks every level is formed from the rank's own band of rows (LocalHierarchy:
    rank-local Galerkin products, level part_levels all-gathered from the ranks' rows).  Fast numerics against the
    one-GPU default: at n >= 72 both apply level 1 matrix-free in one launch (the partition over each rank's owned
    coarse rows and ghost rows, or the replicated level when it is the gather level), below it both the stored level."""
    errfile = str(tmp_path / "err.txt")
    _spawn(_mg_worker, (world, _free_port(), n, inner, min_cells, halo, errfile, numerics), world, errfile)


def _fgmres_worker(rank, world, port, n, inner, maxiter, outdir, errfile, numerics="exact"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from mp_block_preconditioners_amd.distributed import solve_distributed
        iF, iP = _inner_pair(inner)
        res = solve_distributed(n, 1.0, 100.0, 1.0, inner_F=iF, inner_P=iP, tol=1e-8, maxiter=maxiter,
                                mg_min_cells=0, numerics=numerics)
        np.save(os.path.join(outdir, f"x_{rank}.npy"), res["x_local"].cpu().numpy())
        np.save(os.path.join(outdir, f"rows_{rank}.npy"), res["rows"])
        np.save(os.path.join(outdir, f"hist_{rank}.npy"), np.asarray(res["residuals"]))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise


@pytest.mark.parametrize("world,n,inner,maxiter,numerics", [
    (2, 32, (("chebyshev", 4), ("chebyshev", 4)), 40, "exact"), (3, 48, MG1, 60, "exact"), (2, 64, MG1, 60, "exact"),
    (2, 64, MG1, 60, "fast"), (3, 48, MG1, 60, "fast"), (2, 32, (("chebyshev", 4), ("chebyshev", 4)), 40, "fast"),
    (2, 128, MG1, 60, "fast")])
def test_distributed_fgmres_matches_single_gpu(world, n, inner, maxiter, numerics, tmp_path):
    """Row 17: FGMRES (solve.py:285) over the row partition -- the partitioned A, the partitioned preconditioner,
    reproducible inner products reduced over the ranks -- gives the one-GPU solve's residual history and iterate bit
    for bit (the manufactured problem of solve.py:52-80)."""
    import mp_block_preconditioners_amd as mpb
    errfile = str(tmp_path / "err.txt")
    _spawn(_fgmres_worker, (world, _free_port(), n, inner, maxiter, str(tmp_path), errfile, numerics), world, errfile)
    bp = mpb.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    iF, iP = _inner_pair(inner)
    pc = mpb.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP, numerics=numerics)
    _, b = mpb.manufactured_problem(n, 1.0, -1.0, 1.0, 100.0, 1.0)
    hist = []
    x, info = mpb.fgmres(A, torch.from_numpy(b).cuda(), M=pc, tol=1e-8, maxiter=maxiter, residuals=hist)
    x = x.cpu().numpy()
    got = np.zeros_like(x)
    for r in range(world):
        h = np.load(os.path.join(str(tmp_path), f"hist_{r}.npy"))
        assert np.array_equal(h, np.asarray(hist)), (r, len(h), len(hist))
        got[np.load(os.path.join(str(tmp_path), f"rows_{r}.npy"))] = np.load(os.path.join(str(tmp_path), f"x_{r}.npy"))
    assert np.array_equal(got.view(np.uint64), x.view(np.uint64))
    if "mg" in inner[0]:
        assert info == 0


def _comm_worker(_index, port, n, errfile):
    """solve_distributed over the RCCL self-exchange: the partitioned operator A u holds a communicator of its own (its
    eager side-stream exchanges never mix with a preconditioner's graph-replayed ones), the partitioned
    preconditioners of the process group share one (mpbp_halo_create_shared), and the solve with maxiter / restrt left
    at their defaults runs."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=0, world_size=1)
        import mp_block_preconditioners_amd as mpb
        from mp_block_preconditioners_amd.distributed import DistributedSchurPreconditioner, solve_distributed
        res = solve_distributed(n, 1.0, 100.0, 1.0, inner_F=mpb.InnerSolver("mg", 1), inner_P=mpb.InnerSolver("mg", 1),
                                tol=1e-8, self_halo=True, halo="rccl", mg_min_cells=0, keep_operators=True)
        dA, M = res["A"], res["M"]
        assert dA._rccl is not None and M._rccl is not None
        assert dA._rccl.comm != 0 and M._rccl.comm != 0 and dA._rccl.comm != M._rccl.comm
        assert M._rccl.comm_refs == 1 and dA._rccl.comm_refs == 1
        assert res["info"] == 0, (res["info"], len(res["residuals"]))
        M2 = DistributedSchurPreconditioner(n, 1.0, 100.0, 1.0, self_halo=True, halo="rccl")
        assert M2._rccl.comm == M._rccl.comm and M._rccl.comm_refs == 2
        dA.close()
        assert M._rccl.comm_refs == 2
        M2.close()
        assert M._rccl.comm_refs == 1
        M.close()
        dist.destroy_process_group()
    except BaseException as e:
        with open(errfile, "a") as f:
            f.write(f"{type(e).__name__}: {e}\n")
        raise


def test_solve_distributed_communicators(tmp_path):
    errfile = str(tmp_path / "err.txt")
    _spawn(_comm_worker, (_free_port(), 32, errfile), 1, errfile)


def _default_maxiter_worker(rank, world, port, n, outdir, errfile):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import mp_block_preconditioners_amd as mpb
        from mp_block_preconditioners_amd.distributed import solve_distributed
        res = solve_distributed(n, 1.0, 100.0, 1.0, inner_F=mpb.InnerSolver("jacobi", 1),
                                inner_P=mpb.InnerSolver("jacobi", 1), tol=1e-14, maxiter=None)
        assert res["A"].n_own < 200   # the rank-local length is below pyamg's default cap of 200
        np.save(os.path.join(outdir, f"hist_{rank}.npy"), np.asarray(res["residuals"]))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise


def test_distributed_fgmres_default_maxiter(tmp_path):
    """FGMRES's default maxiter / restart come from the GLOBAL length (min(n, 200)), identical on every
    rank -- a rank-local default would leave one rank waiting in an all-reduce -- and equal to the one-GPU solve's."""
    import mp_block_preconditioners_amd as mpb
    n, world = 6, 2
    errfile = str(tmp_path / "err.txt")
    _spawn(_default_maxiter_worker, (world, _free_port(), n, str(tmp_path), errfile), world, errfile)
    bp = mpb.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    pc = mpb.ApproxSchurPreconditioner(F, D, G, inner_F=mpb.InnerSolver("jacobi", 1), inner_P=mpb.InnerSolver("jacobi", 1))
    _, b = mpb.manufactured_problem(n, 1.0, -1.0, 1.0, 100.0, 1.0)
    hist = []
    mpb.fgmres(A, torch.from_numpy(b).cuda(), M=pc, tol=1e-14, residuals=hist)
    for r in range(world):
        h = np.load(os.path.join(str(tmp_path), f"hist_{r}.npy"))
        assert np.array_equal(h, np.asarray(hist)), (r, len(h), len(hist))


def _configs4_worker(rank, world, port, n, errfile, numerics="exact"):
    """configs[4]: the 2048^2 apply row-partitioned over 8 ranks (256 grid rows each: the 8-GPU run's geometry, CA
    ghost depths and halo sizes) on one GPU over gloo, bit for bit against the one-GPU apply."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import mp_block_preconditioners_amd as mpb
        from mp_block_preconditioners_amd.distributed import DistributedSchurPreconditioner
        iF, iP = mpb.InnerSolver("chebyshev", 4), mpb.InnerSolver("chebyshev", 4)
        dpc = DistributedSchurPreconditioner(n, 1.0, 100.0, 1.0, inner_F=iF, inner_P=iP, numerics=numerics)
        assert dpc.ca and dpc.part.L == n // world
        gids = torch.from_numpy(dpc.local_to_global_rows()).cuda()
        v = torch.from_numpy(np.random.default_rng(2048).standard_normal(5 * n * n)).cuda()
        got = dpc.apply(v[gids].contiguous())
        torch.cuda.synchronize()
        dpc.close()
        del dpc
        torch.cuda.empty_cache()
        # the one-GPU reference, one rank at a time (bounds the GPU memory of 8 ranks sharing one card)
        for turn in range(world):
            if turn == rank:
                bp = mpb.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
                _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
                pc = mpb.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP, numerics=numerics,
                                                   kernel_opts={"q13_mf": 0})   # (the stored Gt_F_G, as the partition)
                ref = pc.apply(v)[gids]
                assert torch.equal(got, ref), float((got - ref).abs().max())
                del pc, F, D, G, bp, ref
                torch.cuda.empty_cache()
            dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise


@pytest.mark.parametrize("numerics", ["exact", "fast"])
def test_configs4_2048_over_8_ranks(numerics, tmp_path):
    """BASELINE configs[4] (2048^2, rows partitioned over 8 ranks) on one GPU: every rank's rows of the partitioned
    apply equal the one-GPU apply's, in both numerics (fast: the bench's headline numerics).  The RCCL-over-xGMI
    transport itself needs the 8-GPU node (bench.py --gpus 8)."""
    errfile = str(tmp_path / "err.txt")
    _spawn(_configs4_worker, (8, _free_port(), 2048, errfile, numerics), 8, errfile)
