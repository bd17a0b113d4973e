"""Setup time of the row-partitioned preconditioner (rank-local assembly, DistributedSchurPreconditioner) at configs[4]'s
2048^2 over W gloo ranks that all share one GPU (the 8-GPU geometry rehearsed on one card; the max over ranks is
printed).  Builds run in the order given (--order); the first pays the process's cold start.

    python tools/setup_timing.py [--world 8] [--n 2048] [--inner mg:1] [--global-products]

Each build reports its seconds (max over ranks, per phase) and the peak device memory a rank allocated during it
(torch.cuda.max_memory_allocated, max over ranks): with multigrid inner solves the rank-local hierarchies
(LocalHierarchy) against --global-products' whole operators and hierarchy on every rank.
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, port, n, order, q, keep_cache=False, inner="chebyshev:4", local_products=True, threads=0):
    import torch
    import torch.distributed as dist
    if threads:   # host threads per rank (the ranks share the box's cores)
        torch.set_num_threads(threads)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MPBP_SETUP_TIMING="1")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import mp_block_preconditioners_amd as mpb
    from mp_block_preconditioners_amd.distributed import DistributedSchurPreconditioner
    out = {}
    kind, _, k = inner.partition(":")
    for numerics in order:
        dist.barrier()
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        t0 = time.perf_counter()
        dpc = DistributedSchurPreconditioner(n, 1.0, 100.0, 1.0, inner_F=mpb.InnerSolver(kind, int(k or 4)),
                                             inner_P=mpb.InnerSolver(kind, int(k or 4)), numerics=numerics,
                                             local_products=local_products)
        torch.cuda.synchronize()
        names = sorted(dpc.setup_phases)
        el = torch.tensor([time.perf_counter() - t0, torch.cuda.max_memory_allocated() - base,
                           torch.cuda.memory_allocated() - base] + [dpc.setup_phases[k] for k in names],
                          dtype=torch.float64)
        mine = {"total": round(time.perf_counter() - t0, 4), **{k: round(v, 4) for k, v in dpc.setup_phases.items()}}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        out[f"{len(out) + 1}_{numerics}"] = {"phases_per_rank": per_rank, "total": float(el[0]),
                                             "peak_mem_gb": round(float(el[1]) / 1e9, 3),
                                             "kept_mem_gb": round(float(el[2]) / 1e9, 3), "phases_max_over_ranks": {
            k: round(float(v), 4) for k, v in zip(names, el[3:].tolist())}}
        if rank == 0:   # progress (a silent multi-minute run looks hung to the GPU harness)
            print(json.dumps({"build": len(out), "numerics": numerics, **out[f"{len(out)}_{numerics}"]}), flush=True)
        dpc.close()
        del dpc
        if not keep_cache:
            torch.cuda.empty_cache()
    if rank == 0:
        q.put(out)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--order", default="exact,fast,exact,fast", help="numerics of the successive builds")
    ap.add_argument("--fresh", action="store_true", help="every build in a fresh set of rank processes")
    ap.add_argument("--keep-cache", action="store_true", help="no torch.cuda.empty_cache() between builds")
    ap.add_argument("--inner", default="chebyshev:4", help="both inner solves, kind:k (e.g. mg:1)")
    ap.add_argument("--threads", type=int, default=0, help="torch host threads per rank (0: torch's default)")
    ap.add_argument("--global-products", action="store_true",
                    help="every rank forms the global operators (and multigrid hierarchy) and extracts its rows")
    a = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    order = a.order.split(",")
    res = {}
    for batch in ([[o] for o in order] if a.fresh else [order]):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        q = ctx.Queue()
        procs = [ctx.Process(target=worker, args=(r, a.world, port, a.n, batch, q, a.keep_cache, a.inner,
                                                  not a.global_products, a.threads))
                 for r in range(a.world)]
        for p in procs:
            p.start()
        out = q.get(timeout=600)
        for p in procs:
            p.join(timeout=120)
        for k, v in out.items():
            res[f"{len(res) + 1}_{k.split('_', 1)[1]}"] = v
    print(json.dumps({"n": a.n, "world": a.world, "backend": "gloo, every rank on one GPU",
                      "processes": "a fresh set per build" if a.fresh else "one set for all builds",
                      "empty_cache_between_builds": not a.keep_cache, "inner": a.inner,
                      "products": "global on every rank" if a.global_products else "rank-local",
                      "host_threads_per_rank": a.threads or "torch default",
                      "setup_seconds_max_over_ranks": res,
                      "note": "DistributedSchurPreconditioner construction: rank-local F / D / G rows, commutator "
                              "products of the owned rows, Chebyshev bounds or the multigrid levels, CA ghost "
                              "diagonals, halo plan; memory: peak / kept device bytes a rank allocated during the build"}),
          flush=True)


if __name__ == "__main__":
    main()
