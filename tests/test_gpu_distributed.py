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


def _worker(rank, world, port, n, layout, f_mode, kind, errfile, ca="auto", fuse_g=True):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import mp_block_preconditioners_amd as mpb
        from mp_block_preconditioners_amd.distributed import DistributedSchurPreconditioner
        mpb.lib().mpbp_set_march_rows(kind)
        iF, iP = mpb.InnerSolver("chebyshev", 4), mpb.InnerSolver("chebyshev", 3)
        dpc = DistributedSchurPreconditioner(n, 1.0, 100.0, 1.0, inner_F=iF, inner_P=iP, layout=layout,
                                             f_mode=f_mode, ca=ca, fuse_g=fuse_g)
        assert dpc.fuse_g == bool(fuse_g and dpc.ca)
        assert (dpc.f_stencil is not None) == (f_mode != "assembled")
        if ca is True:
            assert dpc.ca and dpc.h_u == dpc.ca_q + 2 + 1 + 3, (dpc.h_u, dpc.ca_q)
        bp = mpb.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
        _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
        pc = mpb.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP, layout=layout, f_mode="assembled")
        assert (pc.inner_F.lmin, pc.inner_F.lmax) == (dpc.inner_F.lmin, dpc.inner_F.lmax)
        v = torch.from_numpy(np.random.default_rng(5).standard_normal(pc.shape[0])).cuda()
        gids = torch.from_numpy(dpc.local_to_global_rows()).cuda()
        ref = pc.apply(v)[gids]
        for _ in range(2):
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


def _self_halo_worker(_index, port, n, halo, f_mode, pg_mode, kind, graph, errfile, overlap=False, ca="auto",
                      inner=(("chebyshev", 4), ("chebyshev", 3))):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=0, world_size=1)
        import mp_block_preconditioners_amd as mpb
        from mp_block_preconditioners_amd.distributed import DistributedSchurPreconditioner
        mpb.lib().mpbp_set_march_rows(kind)
        iF, iP = mpb.InnerSolver(*inner[0]), mpb.InnerSolver(*inner[1])
        dpc = DistributedSchurPreconditioner(n, 1.0, 100.0, 1.0, inner_F=iF, inner_P=iP, f_mode=f_mode,
                                             pg_mode=pg_mode, halo=halo, self_halo=True, halo_overlap=overlap,
                                             ca=ca)
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
