"""Row-partitioned apply on CPU: world_size 2 (and 3) over gloo, checked bit for bit against the
single-process oracle.  Exercises the product's partition host logic (RowPartition, colmap,
halo_reach, boundary_ranges, HaloExchanger); the arithmetic runs on the oracle's kernels."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

PARAMS = dict(xi=1.0, eta_n=100.0, eta_s=1.0, c=1.0, d_u=-1.0, d_p=1.0, d_div=-1.0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, inners, errfile):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from mp_block_preconditioners_amd.distributed import (HaloExchanger, RowPartition, boundary_ranges,
                                                              halo_reach)
        from oracle.dist_oracle import dist_apply, extract_rows
        from oracle.schur_oracle import Inner, approx_schur_apply, diagonal, gershgorin
        from oracle.stokes_oracle import StokesSystem
        s = StokesSystem(n, **PARAMS)
        part = RowPartition(n, world, rank)
        ru, rp_ = part.owned_rows(4), part.owned_rows(1)

        def reach(M, rows):
            sub = extract_rows(M, rows, np.arange(M.shape[1], dtype=np.int32), M.shape[1])
            return halo_reach(torch.from_numpy(sub.indptr), torch.from_numpy(sub.indices), torch.from_numpy(rows), n)

        h_u = max(1, reach(s.F, ru), reach(s.D, rp_))
        h_p = max(1, reach(s.G, ru), reach(s.GtG, rp_), reach(s.GtFG, rp_))
        assert h_u == 1 and 1 <= h_p <= 3
        cm_u, cm_p = part.colmap(4, h_u), part.colmap(1, h_p)
        nu_ext, np_ext = part.n_ext(4, h_u), part.n_ext(1, h_p)
        loc = dict(F=extract_rows(s.F, ru, cm_u, nu_ext), D=extract_rows(s.D, rp_, cm_u, nu_ext),
                   G=extract_rows(s.G, ru, cm_p, np_ext), GtG=extract_rows(s.GtG, rp_, cm_p, np_ext),
                   GtFG=extract_rows(s.GtFG, rp_, cm_p, np_ext), nu=part.n_owned(4), np=part.n_owned(1),
                   nu_ext=nu_ext, np_ext=np_ext)
        loc["diag_F"] = diagonal(s.F)[ru]
        loc["diag_P"] = diagonal(s.GtG)[rp_]
        # boundary rows are exactly the rows that read a ghost
        for M, own in ((loc["F"], loc["nu"]), (loc["GtFG"], loc["np"])):
            inner, bnd = boundary_ranges(torch.from_numpy(M.indptr), torch.from_numpy(M.indices), own)
            flags = np.zeros(M.shape[0], bool)
            for a, b in bnd:
                flags[a:b] = True
            reads_ghost = np.array([np.any(M.indices[M.indptr[i]:M.indptr[i + 1]] >= own) for i in range(M.shape[0])])
            assert np.array_equal(flags, reads_ghost)
            assert sum(b - a for a, b in inner + bnd) == M.shape[0]
        ex_u = HaloExchanger(part, 4, h_u, "cpu")
        ex_p = HaloExchanger(part, 1, h_p, "cpu")
        v = np.random.default_rng(99).standard_normal(5 * n * n)
        gids = np.concatenate([ru, 4 * n * n + rp_])
        lmaxF = gershgorin(s.F, diagonal(s.F))
        lmaxP = gershgorin(s.GtG, diagonal(s.GtG))
        for kf, sf, kp, spp in inners:
            iF = Inner(kf, sf, lmaxF / 30, lmaxF) if kf == "chebyshev" else Inner(kf, sf)
            iP = Inner(kp, spp, lmaxP / 30, lmaxP) if kp == "chebyshev" else Inner(kp, spp)
            got = dist_apply(loc, ex_u, ex_p, v[gids], iF, iP)
            ref = approx_schur_apply(s.F, s.D, s.G, s.GtG, s.GtFG, v, iF, iP)[gids]
            assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), (kf, sf, kp, spp)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:   # surface the failure to the parent
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {type(e).__name__}: {e}\n")
        raise


@pytest.mark.parametrize("world,n", [(2, 12), (3, 13)])
def test_partitioned_apply_matches_global(world, n, tmp_path, oracle_built):
    errfile = str(tmp_path / "err.txt")
    inners = [("chebyshev", 4, "chebyshev", 3), ("jacobi", 2, "jacobi", 3)]
    try:
        mp.spawn(_worker, args=(world, _free_port(), n, inners, errfile), nprocs=world, join=True)
    except Exception:
        msg = open(errfile).read() if os.path.exists(errfile) else ""
        pytest.fail(f"distributed worker failed:\n{msg}")


def test_row_partition_maps():
    from mp_block_preconditioners_amd.distributed import RowPartition
    n, world, h = 13, 3, 2
    parts = [RowPartition(n, world, k) for k in range(world)]
    assert [p.L for p in parts] == [5, 4, 4] and parts[-1].r1 == n
    for p in parts:
        cm = p.colmap(2, h)
        own = p.n_owned(2)
        assert sorted(cm[cm >= 0].tolist()) == list(range(p.n_ext(2, h)))
        for f in range(2):
            for gr in range(n):
                row = cm[f * n * n + gr * n: f * n * n + (gr + 1) * n]
                d = min((gr - p.r0) % n, (p.r0 - gr) % n, (gr - (p.r1 - 1)) % n, ((p.r1 - 1) - gr) % n)
                if p.r0 <= gr < p.r1:
                    assert np.all((row >= 0) & (row < own))
                elif d <= h:
                    assert np.all(row >= own)
                else:
                    assert np.all(row == -1)
    with pytest.raises(ValueError):
        RowPartition(8, 4, 0).colmap(1, 3)


@pytest.mark.parametrize("n,world,h", [(12, 3, 2), (20, 2, 9), (9, 1, 3), (17, 4, 4)])
def test_ext_rows_inverts_colmap(n, world, h):
    """The ext layout's global ids (ext_rows: the CA schedule's ghost-row diagonals) are the inverse of
    colmap (the extracted operators' column renumbering), ghosts included, for every rank."""
    from mp_block_preconditioners_amd.distributed import RowPartition
    for rank in range(world):
        part = RowPartition(n, world, rank, ghosts=True)
        for nf in (1, 4):
            gid = part.ext_rows(nf, h)
            assert gid.size == part.n_ext(nf, h)
            cm = part.colmap(nf, h)
            own = part.n_owned(nf)
            assert np.array_equal(cm[gid[:own]], np.arange(own))
            if world > 1:   # a ghost row may sit in two slots (2 h > a neighbour's rows): same global id
                assert np.all(cm[gid] >= 0) and np.array_equal(gid[cm[gid]], gid)
            else:           # one rank: the periodic ghosts duplicate owned rows
                assert np.array_equal(np.sort(np.unique(gid)), np.arange(nf * n * n))


def test_host_staged_halo_failure_is_raised():
    """a host-staged (torch / gloo) exchange that fails inside the C apply is latched by the callback (ctypes
    would swallow it) and raised by _Halos.check(), which DistributedSchurPreconditioner.apply calls after every apply;
    the latch is cleared so a later apply runs its exchanges again."""
    from mp_block_preconditioners_amd import _lib
    from mp_block_preconditioners_amd.distributed import _Halos

    class Boom:
        calls = 0

        def begin(self, x):
            Boom.calls += 1
            raise OSError("peer went away")

        def end(self, x):
            pass

    h = _Halos("torch", None, None, "cpu")
    h._ex[0] = Boom()
    x = torch.zeros(8, dtype=torch.float64)
    h.register(x)
    h.fn(None, 0, x.data_ptr(), _lib.HALO_BEGIN, None)
    h.fn(None, 0, x.data_ptr(), _lib.HALO_BEGIN, None)   # latched: no second attempt inside the same apply
    assert Boom.calls == 1
    with pytest.raises(RuntimeError, match="peer went away"):
        h.check()
    h.check()                                             # cleared
    h.fn(None, 0, x.data_ptr(), _lib.HALO_BEGIN, None)
    assert Boom.calls == 2


def test_row_partition_error_message():
    from mp_block_preconditioners_amd.distributed import RowPartition
    with pytest.raises(ValueError, match=">= 1 row"):
        RowPartition(4, 2, 0, bounds=((0, 4), (4, 0)))
    with pytest.raises(ValueError, match=">= 0 rows"):
        RowPartition(4, 2, 0, bounds=((0, 4), (5, 0)), allow_empty=True)
