"""Benchmark: preconditioner applies per second on the multiphase-Stokes system on MI355X, with the roofline
of the dominant kernel and the CPU oracle timed beside it.

One step = one application of the approximate-commutator block preconditioner (solve.py:257-277,
``mpbp_schur_apply``) to a resident random vector of 5 n^2 doubles.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--grid n] [--weak] ...

N = 1: BASELINE configs[2], the 1024^2 grid on one GPU.  N > 1: BASELINE configs[4], the 2048^2 grid row-
partitioned over N ranks (one per GPU, RCCL point-to-point halos).  `python bench.py --gpus N` launches the N
ranks itself (a torch.distributed.run child process started before anything touches the GPU); under an
external launcher (WORLD_SIZE set) --gpus must equal WORLD_SIZE.  `value` counts applies of the global system
in 1024^2-cell equivalents (applies/s x n^2 / 1024^2: exactly applies/s at N = 1), so the N = 1 and N > 1
lines share a unit.  --weak instead grows the grid as n = round(1024 sqrt(N)).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0    # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
_KEEP_ALIVE = []         # objects whose lifetime must span the run (an installed kernel_options scope)
MG_KW = {}               # --mg-coarsest: InnerSolver keyword arguments of every multigrid inner solve the run builds


def parse_inner(s):
    kind, _, k = s.partition(":")
    return kind, int(k or 4)


def sweep_bytes(pc, layout, kind, sweeps, fused_init, f_tile=False, f_solve=False):
    """Algorithmic HBM bytes of the F inner-solve launches bench.py times: one (bytes, solve) per recorded launch of
    one apply, in record order, and the kernel's name.

    mpbp_schur_apply records events around the launches of sweeps s = 1 .. K-1 of both F solves (s = 2 .. K-1 when the
    init pass is fused into sweep 1).  A sweep moves per F row: x_in, b, x_out (8 B each), the direction d read
    (Chebyshev) and written (Chebyshev, not on the last sweep), the solve's `sub` on the second solve's last sweep, and
    diag (assembled layouts); plus the matrix (assembled: 12 B per entry + index data) or the thn tables (matrix-free:
    cell, u-face, v-face = 3 x 8 B per cell = 6 B per row).  With G x_p recomputed in the second solve (fuse_g), its
    sweeps read x_p (8 B per cell = 2 B per row) instead of b.  Tolerance-mode F solves of >= 4 sweeps run their last
    two sweeps as ONE launch (k_march2): x_in, b, d_in read and x_out written once for the pair (x_s stays in LDS).
    f_solve (one GPU, tolerance mode, 3 or 4 updates): each whole F solve is ONE launch (k_fsolve) reading b (or x_p),
    the thn tables (and the second solve's sub) and writing x once."""
    F = pc.F
    nF, nnzF = F.shape[0], F.nnz
    cheb = kind == "chebyshev"
    stencil = getattr(pc, "f_stencil", None) is not None
    fast = getattr(pc, "numerics", "exact") == "fast"
    pair = stencil and fast and cheb and fused_init and sweeps >= 4
    if stencil:
        prm = pc.f_stencil.prm   # the parameter identities compiled into the F policy (csrc: with_f_identities)
        n_f = int(prm.n)
        pow2 = (n_f & (n_f - 1)) == 0
        pol = ("FStencilDevM<7>" if prm.eta_n == 1.0 else ("FStencilDevM<13>" if pow2 else "FStencilDevM<5>")) \
            if (prm.d_u == -1.0 and prm.eta_s == 1.0) else "FStencilDev"
        if fast:
            pol = "FStencilFast"
        fixed, kname = 3 * 8 * (nF // 4), f"k_march<{pol}, XPlain, EpiCheb> (F sweep, matrix-free)"
        if pair:
            kname = ("k_ftile<pair> (the F solve's last two Chebyshev sweeps in one launch on 64 x 8 tiles, "
                     "matrix-free, tolerance mode)" if f_tile else
                     "k_march2<FStencilFast> (the F solve's last two Chebyshev sweeps in one marching launch, "
                     "matrix-free, tolerance mode)")
    elif layout == "sell":
        fixed = nnzF * 12 + nF * 1 + pc.sell_of("F").nslices * 16
        kname = "k_sell_rows<EpiCheb> (F sweep, SELL-64)"
    else:
        fixed, kname = nnzF * 12 + (nF + 1) * 4 + F.blocks.count * 8, "k_csr_wave<EpiCheb> (F sweep, CSR)"
    fuse_g = bool(getattr(pc, "fuse_g", False))
    out = []
    if stencil and fast and cheb and f_solve:
        w = int(getattr(getattr(pc, "kernel_opts", None), "f_solve_tile", 0)) == 1
        kname = ("%s (a whole F Chebyshev solve -- x0 and %d sweeps -- in one launch on %s tiles, matrix-free, "
                 "tolerance mode)" % ("k_fsolve_w" if w else "k_fsolve", sweeps - 1, "32 x 16" if w else "64 x 8"))
        for solve in (1, 2):
            gx = fuse_g and solve == 2
            rhs = nF // 4 * 8 if gx else nF * 8            # x_p (one field) or b (four)
            out.append((fixed + rhs + nF * 8 + (nF * 8 if solve == 2 else 0), solve))
        return out, kname
    for solve in (1, 2):
        s = 2 if fused_init else 1
        while s < sweeps:
            pr = pair and s == sweeps - 2
            last = s == sweeps - 1 or pr
            gx = fuse_g and solve == 2                              # b = G x_p recomputed: x_p, 8 B per cell
            streams = 3 + (0 if stencil else 1) - (1 if gx else 0)  # x_in, b, x_out (+ diag)
            streams += (1 + (0 if last else 1)) if cheb else 0      # d read (+ write)
            streams += 1 if (last and solve == 2) else 0            # sub
            out.append((fixed + nF * 8 * streams + (nF // 4 * 8 if gx else 0), solve))
            s += 2 if pr else 1
    return out, kname


def roofline_of(per_apply, sweep_ms, solve):
    """Mean algorithmic bytes, mean HIP-event duration (s) and launch count of the recorded sweeps of one solve."""
    if not per_apply or not sweep_ms:
        return float("nan"), float("nan"), 0
    sel = [(per_apply[i % len(per_apply)][0], ms) for i, ms in enumerate(sweep_ms)
           if per_apply[i % len(per_apply)][1] == solve]
    if not sel:
        return float("nan"), float("nan"), 0
    return (sum(b for b, _ in sel) / len(sel), sum(ms for _, ms in sel) / len(sel) / 1e3, len(sel))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default WORLD_SIZE or 1.  Without WORLD_SIZE, N > 1 launches N ranks")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--grid", "--grid-n", dest="n", type=int, default=None,
                    help="global grid size n (n x n cells); default 1024 at N = 1 (configs[2]), 2048 at N > 1 "
                         "(configs[4])")
    ap.add_argument("--weak", action="store_true", help="weak scaling: global grid round(1024 sqrt(N))")
    ap.add_argument("--strong", action="store_true", help="(kept for old command lines) same as the default")
    ap.add_argument("--xi", type=float, default=1.0)
    ap.add_argument("--eta-n", type=float, default=100.0)
    ap.add_argument("--eta-s", type=float, default=1.0)
    ap.add_argument("--inner-f", default="chebyshev:4")
    ap.add_argument("--inner-p", default="chebyshev:4")
    ap.add_argument("--layout", default="sell", choices=["sell", "csr"])
    ap.add_argument("--numerics", default="fast", choices=["fast", "exact"],
                    help="matrix-free F rows: 'fast' (tolerance mode, FMA-contracted, reciprocal diagonals: within 1e-12 "
                         "of the oracle, north_star's fp64 bar) or 'exact' (the assembly's IEEE operations: bit-identical "
                         "to the oracle)")
    ap.add_argument("--f-mode", default="auto", choices=["auto", "stencil", "assembled"],
                    help="F sweeps: recompute F from thn (stencil) or stream the assembled F")
    ap.add_argument("--pg-mode", default="auto", choices=["auto", "stencil", "assembled"],
                    help="D, G, Gt_G: recompute from thn (stencil) or stream the stored operators")
    ap.add_argument("--q-mode", default="auto", choices=["auto", "diamond", "assembled"],
                    help="Gt_F_G: values in the 13-point diamond layout (columns implicit) or the assembled copy")
    ap.add_argument("--march-rows", type=int, default=0,
                    help="grid rows per workgroup of the marching stencil kernels (matrix-free F, D, G, Gt_G); "
                         "0: the count that fills one round of workgroups per launch")
    ap.add_argument("--pg-direct", type=int, default=None, help="1: D / Gt_G sweeps as one thread per cell (no LDS)")
    ap.add_argument("--f-pair", type=int, default=None,
                    help="fast numerics: 1 (default) runs an F solve's last two sweeps as one k_march2 launch, 0 as two")
    ap.add_argument("--f-direct", type=int, default=None,
                    help="fast numerics: 1 runs the single F sweeps on the direct kernel (one thread per cell, no LDS)")
    ap.add_argument("--f-tile", type=int, default=None,
                    help="fast numerics: 1 (default) runs an F solve's x0 + first sweep and its last pair on 2D tiles, "
                         "0 on the marching kernels")
    ap.add_argument("--f-solve", type=int, default=None,
                    help="fast numerics: 1 (default) runs each F solve of 3 or 4 updates as one k_fsolve launch, "
                         "0 as k_ftile launches")
    ap.add_argument("--solve-numerics", default=None, choices=["fast", "exact"],
                    help="N > 1: numerics of the partitioned multigrid apply and the distributed FGMRES section "
                         "(default: --numerics)")
    ap.add_argument("--q13-sym", type=int, default=None,
                    help="fast numerics: 1 (default) reads Gt_F_G's diamond upper half only (symmetric product); 0: all 13")
    ap.add_argument("--gtg-drhs", type=int, default=None,
                    help="1 (default): the first fused Gt_G solve builds rhs = D Finv_v + v_p itself; 0: a D launch")
    ap.add_argument("--gtg-fused", type=int, default=None,
                    help="1 (default): each Chebyshev Gt_G solve as one tiled launch; 0: one launch per sweep")
    ap.add_argument("--mg-galerkin-mf", type=int, default=None,
                    help="fast numerics: 2 (default) applies the F hierarchy's level 1 as R0 (F (P0 x)) in one k_gal1 "
                         "launch, 1 in three launches, 0 streams its stored Galerkin matrix")
    ap.add_argument("--mg-galerkin-mf-p", type=int, default=None,
                    help="fast numerics: 1 (default) applies the pressure hierarchy's level 1 as R0 (Gt_G (P0 x)) "
                         "(one k_gal1p launch with --mg-galerkin-mf 2), 0 streams its stored Galerkin matrix")
    ap.add_argument("--svl-min-rows", type=int, default=None,
                    help="multigrid levels above this many rows get a stencil-values copy (mg.SVL_MIN_ROWS; -1: none)")
    ap.add_argument("--stored-transfers", action="store_true",
                    help="multigrid transfers from their stored forms instead of matrix-free")
    ap.add_argument("--mg-group-rows", type=int, default=None,
                    help="multigrid levels / transfers with at most this many rows on the grouped CSR kernel (0: off)")
    ap.add_argument("--no-fuse-g", action="store_true",
                    help="launch G x_p separately instead of recomputing it inside the second F solve's sweeps")
    ap.add_argument("--no-ca", action="store_true",
                    help="row partition: exchange before every sweep instead of the communication-avoiding schedule")
    ap.add_argument("--self-halo", action="store_true",
                    help="N = 1 only: run the row-partitioned apply with the ghost rows refreshed by the periodic "
                         "self-exchange over RCCL (measures the multi-GPU code path's overhead on one GPU)")
    ap.add_argument("--halo-overlap", action="store_true",
                    help="RCCL halo group on a side stream overlapping the interior rows (default: in order)")
    ap.add_argument("--kernel-opt", action="append", default=[], metavar="NAME=VALUE",
                    help="a kernel choice (mpbp_kernel_opts field) for every plan of the run; repeatable")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-spmv", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="launch the apply eagerly instead of a hipGraph")
    ap.add_argument("--no-check", action="store_true", help="N > 1: skip the bit-exact check against one GPU")
    ap.add_argument("--no-mg", action="store_true",
                    help="skip the multigrid apply section (mg:1 / mg:1 applies/s and its dominant kernel's roofline)")
    ap.add_argument("--no-solve", action="store_true",
                    help="skip the solve-level section (FGMRES to 1e-8 on the manufactured problem, N = 1)")
    ap.add_argument("--partitioned-graph", action="store_true",
                    help="(kept for old command lines: the default for RCCL ranks)")
    ap.add_argument("--global-products", action="store_true",
                    help="N > 1: every rank forms the whole Gt_G / Gt_F_G (the default forms its own pressure rows)")
    ap.add_argument("--eager-partitioned", action="store_true",
                    help="N > 1: launch the partitioned apply eagerly instead of replaying its hipGraph")
    ap.add_argument("--mg-coarsest", type=int, default=None,
                    help="multigrid sections: coarsening stops at n <= this (InnerSolver.coarsest; default 16)")
    ap.add_argument("--detail-json", default=None, metavar="PATH",
                    help="also write the full record (every note and timing description) to PATH; stdout keeps the "
                         "compact line")
    args = ap.parse_args()

    # --gpus N > 1 without a launcher: start the N ranks as a child process BEFORE anything touches the GPU
    # (torch is not even imported yet) and exit with its status; never re-exec this process
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        return launch_ranks(args.gpus)
    if env_world is not None and args.gpus is not None and int(env_world) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={env_world} set by the launcher")

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MPBP_BENCH_BACKEND=gloo rehearses the N > 1 path with several ranks on one GPU (ghosts staged
    # through host memory); the measured configuration is RCCL ("nccl"), one GPU per rank.
    backend = os.environ.get("MPBP_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if world > 1 and backend == "nccl" and ndev < world:
        raise SystemExit(f"bench.py: {world} RCCL ranks need {world} GPUs, this node shows {ndev} "
                         "(MPBP_BENCH_BACKEND=gloo rehearses several ranks on one GPU)")
    dev_index = local % max(1, ndev)
    torch.cuda.set_device(dev_index)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
    elif args.self_halo:
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{29400 + os.getpid() % 1000}", rank=0,
                                world_size=1, **({"device_id": torch.device("cuda", dev_index)} if backend == "nccl" else {}))
    partitioned = world > 1 or args.self_halo

    import mp_block_preconditioners_amd as mp
    from mp_block_preconditioners_amd._lib import check as _check, lib as _lib
    _check(_lib().mpbp_set_march_rows(args.march_rows))
    if args.pg_direct is not None:
        _check(_lib().mpbp_set_pg_direct(args.pg_direct))
    if args.f_pair is not None:
        _check(_lib().mpbp_set_f_pair(args.f_pair))
    if args.f_direct is not None:
        _check(_lib().mpbp_set_f_direct(args.f_direct))
    if args.f_tile is not None:
        _check(_lib().mpbp_set_f_tile(args.f_tile))
    if args.gtg_fused is not None:
        _check(_lib().mpbp_set_gtg_fused(args.gtg_fused))
    if args.f_solve is not None:
        _check(_lib().mpbp_set_f_solve(args.f_solve))
    if args.gtg_drhs is not None:
        _check(_lib().mpbp_set_gtg_drhs(args.gtg_drhs))
    if args.q13_sym is not None:
        _check(_lib().mpbp_set_q13_sym(args.q13_sym))
    if args.mg_galerkin_mf is not None:
        _check(_lib().mpbp_set_mg_galerkin_mf(args.mg_galerkin_mf))
    if args.mg_galerkin_mf_p is not None:
        _check(_lib().mpbp_set_mg_galerkin_mf_p(args.mg_galerkin_mf_p))
    if args.stored_transfers:
        _check(_lib().mpbp_set_mg_mf_transfer(0))
    if args.mg_group_rows is not None:
        _check(_lib().mpbp_set_mg_group_rows(args.mg_group_rows))
    if args.svl_min_rows is not None:
        from mp_block_preconditioners_amd import mg as _mg
        _mg.SVL_MIN_ROWS = None if args.svl_min_rows < 0 else args.svl_min_rows
    if args.kernel_opt:   # this thread's kernel choices for the whole run: every plan made from here starts from them
        from mp_block_preconditioners_amd._lib import kernel_options
        ko = kernel_options(**{k: int(v) for k, v in (o.split("=", 1) for o in args.kernel_opt)})
        ko.__enter__()
        _KEEP_ALIVE.append(ko)

    if args.mg_coarsest is not None:
        MG_KW["coarsest"] = args.mg_coarsest
    if args.weak:
        n = int(round((args.n or 1024) * math.sqrt(world)))
    else:
        n = args.n or (1024 if world == 1 else 2048)
    kf, sf = parse_inner(args.inner_f)
    kp, spp = parse_inner(args.inner_p)
    iF, iP = mp.InnerSolver(kf, sf), mp.InnerSolver(kp, spp)
    A = None
    mg_ops = None
    t_setup = time.perf_counter()
    if not partitioned:
        bp = mp.MultiphaseBlockPreconditioner(n, args.xi, args.eta_n, args.eta_s)
        A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
        pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP, layout=args.layout,
                                          f_mode=args.f_mode, pg_mode=args.pg_mode, q_mode=args.q_mode,
                                          fuse_g=not args.no_fuse_g, numerics=args.numerics)
        mg_ops = (F, D, G) if not args.no_mg else None
        del F, D, G
    else:
        from mp_block_preconditioners_amd.distributed import DistributedSchurPreconditioner
        pc = DistributedSchurPreconditioner(n, args.xi, args.eta_n, args.eta_s, inner_F=iF, inner_P=iP,
                                            layout=args.layout, f_mode=args.f_mode, pg_mode=args.pg_mode,
                                            self_halo=args.self_halo, halo_overlap=args.halo_overlap,
                                            ca=False if args.no_ca else "auto", fuse_g=not args.no_fuse_g,
                                            local_products=not args.global_products, numerics=args.numerics)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup   # assembly, products, layouts, halo plans (the partitioned: per rank)
    _progress(rank, f"setup {setup_s:.1f} s")
    gen = torch.Generator(device="cuda").manual_seed(1234 + rank)
    v = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda", generator=gen)
    out = torch.empty_like(v)
    torch.cuda.synchronize()

    # The apply is captured once into a hipGraph and replayed (one GPU: 14 launches -> 1; N > 1 RCCL ranks: the
    # gather kernels and RCCL point-to-point groups of the halo exchanges are recorded into the graph too, after
    # one eager apply has opened the neighbour connections).  The gloo rehearsal launches eagerly (its halo is
    # host-staged collectives between kernels, which a graph cannot hold).  The timed loop
    # records no events; the F-sweep durations for the roofline come from HIP events that
    # mpbp_schur_apply records around every F sweep on the apply stream, in an eager pass of the same K
    # applies.  That pass and (N = 1) the A u SpMV section run BEFORE the W warmup applies and the timed loop:
    # the GPU then enters the timed loop at its sustained clocks, as inside a solver loop (with nothing before the
    # 5 warmup applies the 20 timed ones read ~9 % lower: the clocks ramp over ~35 ms of load,
    # profiles/r03w_warmup_sc1_ab.jsonl).
    sweeps_per_apply = 2 * max(sf - 1, 0)
    # N > 1: the eager applies/s first, before any capture is attempted -- a capture that fails (or never returns) on a
    # node where the RCCL point-to-point path was never run still leaves this number
    eager_rate = None
    if world > 1:
        dte = timed_loop(lambda: pc.apply(v, out), args.steps, args.warmup, world, dist, torch)
        eager_rate = args.steps / dte * (n * n / float(1024 * 1024))
    graph, graph_note = None, None
    # partitioned applies are captured for the one-GPU self-exchange (bit-exact) and for N > 1 RCCL ranks
    # (default; --eager-partitioned opts out); the side-stream overlap option cannot be captured
    use_graph = not args.no_graph and (not partitioned or (world == 1 and not args.halo_overlap) or
                                       (not args.eager_partitioned and not args.halo_overlap and backend == "nccl"))
    if use_graph:
        if partitioned:   # open the RCCL neighbour connections outside the capture
            pc.apply(v, out)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
        try:
            graph = pc.capture(v, out)
        except Exception as e:   # fall back to eager launches, and say so in the JSON line
            graph, graph_note = None, f"graph capture failed: {e}"
    # untimed GPU sections first: the A u SpMV roofline, then the profiling pass (HIP events around the F sweeps)
    spmv = None
    if A is not None and not args.no_spmv:
        spmv = spmv_bench(A, gen)
        _progress(rank, "spmv section done")
    pc.enable_profiling(max(1, args.steps * sweeps_per_apply))
    pc.reset_profiling()
    for _ in range(args.steps):
        pc.apply(v, out)
    torch.cuda.synchronize()
    sweep_ms = pc.profiled_ms()
    pc.disable_profiling()
    for _ in range(args.warmup):
        graph.replay() if graph is not None else pc.apply(v, out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        graph.replay() if graph is not None else pc.apply(v, out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    launch = "hipgraph" if graph is not None else "eager"

    # N > 1: every rank compares its rows of the partitioned apply with the one-GPU apply of the global
    # system (built on its own GPU from the same operators), bit for bit; plus an order-free checksum of
    # the global output (sum of the results' bit patterns mod 2^64) that the gloo rehearsal can match
    single = None
    if world > 1 and not args.no_check:
        single = single_gpu_check(pc, n, args, iF, iP, rank, dist, torch)
        _progress(rank, f"single-GPU check: bit_exact {single['bit_exact']}")
    psolve = None
    if world > 1 and not args.no_solve:
        if graph is not None:
            del graph
            graph = None
        try:
            psolve = partitioned_solver_section(args, n, rank, world, dist, torch, backend)
        except Exception as e:   # reported, never fatal to the headline line
            psolve = {"error": f"{type(e).__name__}: {e}"}

    # dominant kernel: the fused Chebyshev-Jacobi sweep over F
    fused_init = getattr(pc, "f_stencil", None) is not None and (not partitioned or pc.ca)
    # the dominant kernel's roofline over the first F solve's plain sweeps (b streamed; 192.9 and 159.4 MB, mean
    # 176.2 MB per launch at 1024^2); the second solve's sweeps (G x_p recomputed when fused) are reported beside it
    # (csrc: the tiled F kernels need n >= 76 on one GPU; below that, or with --f-tile 0, the marching ones run)
    f_tile = (args.f_tile is None or args.f_tile != 0) and n >= 76 and not partitioned
    # (csrc fsolve_ok: 3 or 4 updates, n >= 72; else the k_ftile / marching launches)
    # (one GPU, or a row partition on the communication-avoiding schedule: its solves run k_fsolve over owned + ghost rows)
    f_solve = (args.f_solve is None or args.f_solve != 0) and (not partitioned or bool(getattr(pc, "ca", False))) and \
        ((sf == 4 and n >= 72) or (sf == 3 and n >= 70))
    per_apply, kname = sweep_bytes(pc, args.layout, kf, sf, fused_init, f_tile, f_solve)
    sbytes, avg_sweep_s, n_timed = roofline_of(per_apply, sweep_ms, 1)
    achieved = sbytes / avg_sweep_s / 1e9
    gbytes, g_s, g_timed = roofline_of(per_apply, sweep_ms, 2)

    # HBM bytes per F sweep from the committed rocprofv3 PMC passes (tools/pmc_sweep.py +
    # tools/pmc_reduce.py: FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 correction + WRITE_SIZE)
    traffic = None
    spmv_traffic = None
    pmc_files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic_r*.json")))
    if pmc_files and not partitioned:
        try:
            with open(pmc_files[-1]) as f:
                pm = json.load(f)
            key = ("fsolve" if f_solve else "stencil") if getattr(pc, "f_stencil", None) is not None else args.layout
            if int(pm.get("n", -1)) == n and key in pm:
                traffic = pm[key]["traffic_bytes_corrected"]
            if spmv is not None and int(pm.get("n", -1)) == n and "csr_spmv_A" in pm:
                spmv_traffic = pm["csr_spmv_A"]["traffic_bytes_corrected"]
        except (OSError, ValueError, KeyError):
            traffic = None

    # the LinearOperator boundary with host buffers (solve.py:281: pyamg on the host hands M a numpy
    # vector): H2D of v + apply + D2H of the result per call.  Reported beside `value`, never as it.
    host_io = None
    if rank == 0 and not partitioned:
        vh = v.cpu().numpy()
        pc.matvec(vh)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = 10
        for _ in range(reps):
            pc.matvec(vh)
        el = time.perf_counter() - t0
        host_io = {"value": reps / el, "unit": "applies/s",
                   "note": f"ApproxSchurPreconditioner.matvec on a host ndarray ({vh.nbytes / 1e6:.0f} MB in and "
                           "out over PCIe per call through page-locked staging buffers), eager apply; wall clock over 10 calls"}

    mg_apply = None
    if rank == 0 and not partitioned and mg_ops is not None and kf != "mg":
        try:
            mg_apply = mg_apply_bench(*mg_ops, args.steps, args.warmup, gen, numerics=args.numerics)
            _progress(rank, "mg apply section done")
        except Exception as e:   # reported, never fatal to the headline line
            mg_apply = {"error": f"{type(e).__name__}: {e}"}
    mg_ops = None

    cpu = None
    if rank == 0 and not partitioned and not args.no_cpu_baseline:
        cpu = cpu_baseline(pc, v, args.cpu_seconds, kf, sf, kp, spp, args.numerics)
        _progress(rank, "cpu baseline done")

    solve = None
    if rank == 0 and not partitioned and not args.no_solve:
        solve = solve_level(args)

    if rank == 0:
        scale = n * n / float(1024 * 1024)
        value = args.steps / dt * scale
        cfg = "configs[2]" if (world == 1 and n == 1024) else "configs[4]" if n == 2048 else "custom grid"
        line = {
            "metric": "precond-applies/sec",
            "value": value,
            "unit": "applies/s (1024^2-cell equivalents)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: reference operator (thn = 0.25 sin sin + 0.5), random input vector",
            "config": {"workload": f"{n}x{n} MAC grid, approx-commutator Schur preconditioner apply (BASELINE "
                                   f"{cfg}" + (")" if world == 1 else f", rows partitioned over {world} ranks)"),
                       "applies_per_s_of_this_grid": args.steps / dt,
                       "setup_seconds": setup_s,
                       **({"commutator_products": "rank-local rows" if getattr(pc, "local_products", False)
                           else "global"} if world > 1 else {}),
                       "n": n, "unknowns": 5 * n * n, "xi": args.xi, "eta_n": args.eta_n,
                       "eta_s": args.eta_s, "inner_F": f"{kf}:{sf}", "inner_P": f"{kp}:{spp}",
                       "parallelism": f"rows{world}" if world > 1 else "single", "layout": args.layout,
                       "f_sweeps": f"matrix-free-march{args.march_rows or '-auto'}" if getattr(pc, "f_stencil", None) is not None
                       else "assembled",
                       "f_numerics": args.numerics + (" (tolerance mode: FMA-contracted rows, reciprocal diagonals; "
                                                      "<= 1e-12 relative inf-norm vs the oracle)" if args.numerics == "fast"
                                                      else " (bit-identical to the oracle)"),
                       "d_g_gtg": "matrix-free" if getattr(pc, "pg_stencil", None) is not None else "assembled",
                       "gt_f_g": "diamond-13" if getattr(pc, "q13", None) is not None else args.layout,
                       "g_x_p": "recomputed in the second F solve" if getattr(pc, "fuse_g", False) else "kernel",
                       "launch": launch,
                       "before_timed_loop": ("the A u SpMV section, " if spmv is not None else "") +
                                            "the eager profiling pass (K applies), then W warmup applies",
                       **({"halo": f"{pc.halo_impl} ({'self-exchange' if world == 1 else 'neighbour'})",
                           "halo_schedule": (f"communication-avoiding: 2 exchanges per apply, ghost depth "
                                             f"{pc.h_u} (velocity) / {pc.h_p} (pressure)") if pc.ca
                           else "one exchange per sweep"}
                          if partitioned else {}),
                       **({"backend": backend} if world > 1 else {}),
                       **({"note": graph_note} if graph_note else {})},
            **({"bit_exact_vs_single_gpu": single["bit_exact"], "single_gpu_check": single} if single else {}),
            **({"eager_applies_per_s": eager_rate,
                "eager_note": "the same apply launched eagerly, timed (barrier + max over ranks) before any graph "
                              "capture is attempted"} if eager_rate is not None else {}),
            **(psolve or {}),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname,
                         "bytes_per_launch": sbytes, "avg_launch_us": avg_sweep_s * 1e6,
                         "launches_timed": n_timed,
                         "timing": ("HIP events around the first F solve's launch" if f_solve else
                                    "HIP events around each plain sweep of the first F solve")
                                   + " on the apply stream, eager pass of the same K applies after the timed loop",
                         "events": EVENT_NOTE,
                         **({"note": "the whole solve is one launch: b, thn and faces read and x written once (HBM "
                                     "bytes a third of the two-launch path's 285.6 MB), so the kernel is bound by fp64 "
                                     "VALU issue, not HBM -- its SQ counters are in profiles/ (DESIGN.md section 4)"}
                            if f_solve else {})},
            "roofline_second_f_solve": {
                "bound": "hbm", "achieved": gbytes / g_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": gbytes / g_s / 1e9 / HBM_PEAK_GBS, "bytes_per_launch": gbytes, "avg_launch_us": g_s * 1e6,
                "launches_timed": g_timed,
                "kernel": kname + (" with G x_p recomputed per row (x_p read instead of W)"
                                   if getattr(pc, "fuse_g", False) else "")},
            "spmv_A": spmv,
            # north_star's CSR SpMV target: the plain A u product (apply.py:72) on the scipy CSR arrays
            "roofline_csr_spmv": None if spmv is None else {
                "bound": "hbm", "achieved": spmv["csr_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": spmv["csr_gbs"] / HBM_PEAK_GBS, "traffic": spmv_traffic,
                "kernel": "k_csr_wave<EpiStore> (A u, 5N rows, CSR; LDS-DMA staging)",
                "bytes_per_launch": spmv["csr_bytes"], "avg_launch_us": spmv["csr_us"],
                "back_to_back_us": spmv["csr_us_graph"], "frac_back_to_back": spmv["csr_gbs_graph"] / HBM_PEAK_GBS,
                "same_run_stream": spmv.get("calibration"),
                "frac_of_measured_stream": (spmv["csr_gbs"] / spmv["calibration"]["spmv_shape"]["gbs"]
                                            if spmv.get("calibration") else None),
                "timing": spmv.get("timing", "") + " (one kernel per matvec)", "events": EVENT_NOTE},
            "mg_apply": mg_apply,
            "host_buffer_matvec": host_io,
            "solve_level": solve,
            "time_to_solution": time_to_solution(solve, n),
            "cpu_baseline": cpu,
        }
        if args.detail_json:   # the verbose record (every note and timing description) beside the printed line
            with open(args.detail_json, "w") as f:
                json.dump(line, f, indent=1)
        print(json.dumps(compact_line(line)), flush=True)
    if partitioned:
        pc.close()
        dist.destroy_process_group()


def time_to_solution(solve, n):
    """The keyed figure beside the headline: the fastest converged FGMRES solve to 1e-8 of solve_level on this grid
    (the reference's manufactured problem, eta_n = 100 and the stiff 1e4), seconds per solve (the fgmres call)."""
    runs = solve.get("runs") if isinstance(solve, dict) else solve
    out = {}
    for eta in (100.0, 1e4):
        ok = [r for r in (runs or []) if r.get("n") == n and r.get("eta_n") == eta and r.get("converged")]
        if ok:
            b = min(ok, key=lambda r: r["seconds"])
            out[f"eta_n_{eta:g}"] = {"seconds": b["seconds"], "preconditioner": b["preconditioner"],
                                     "iterations": b["iterations"], "apply_ms": b.get("apply_ms"),
                                     "true_rel_residual": b.get("true_rel_residual")}
    return out or None


def _r(x, nd=4):
    """A float rounded to nd significant digits (the printed line's precision; the detail file keeps every digit)."""
    if isinstance(x, float) and math.isfinite(x) and x != 0.0:
        return float(f"{x:.{nd}g}")
    return x


def _roof(r, keep=()):
    """A roofline object without its prose: the contract's fields plus the kernel, bytes and launch time."""
    if not isinstance(r, dict):
        return r
    out = {k: _r(r[k]) if k in ("achieved", "frac", "avg_launch_us") else r[k]
           for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "bytes_per_launch",
                     "avg_launch_us", "launches_timed", "launches_per_apply", *keep) if k in r}
    if isinstance(out.get("kernel"), str):   # the template instance and its one-line role, not the paragraph
        out["kernel"] = out["kernel"].split(" (")[0]
    if isinstance(out.get("traffic"), float):
        out["traffic"] = round(out["traffic"])
    return out


def compact_line(line):
    """The printed JSON line: the contract's keys first, every section without prose, null fields dropped, and
    north_star's CSR SpMV target (roofline_csr_spmv) LAST -- so the whole line, and that object in any case, stays
    inside the last 8 KB of stdout that the driver records.  --detail-json writes the full record."""
    out = {k: v for k, v in line.items() if k not in (
        "roofline", "roofline_second_f_solve", "spmv_A", "roofline_csr_spmv", "mg_apply", "host_buffer_matvec",
        "solve_level", "time_to_solution", "cpu_baseline")}
    cfg = dict(out.get("config") or {})
    cfg.pop("before_timed_loop", None)
    if isinstance(cfg.get("f_numerics"), str):
        cfg["f_numerics"] = cfg["f_numerics"].split(" (")[0]
    out["config"] = cfg
    out["roofline"] = _roof(line.get("roofline"))
    if line.get("roofline") and line["roofline"].get("timing"):
        out["roofline"]["timing"] = "HIP events on the apply stream around each whole-F-solve launch (eager pass, K applies)"
    r2 = line.get("roofline_second_f_solve")
    if isinstance(r2, dict) and r2.get("launches_timed"):
        out["roofline_second_f_solve"] = {"frac": _r(r2["frac"]), "bytes_per_launch": r2["bytes_per_launch"],
                                          "avg_launch_us": _r(r2["avg_launch_us"])}
    out["cpu_baseline"] = line.get("cpu_baseline")
    if isinstance(out["cpu_baseline"], dict):
        cb = dict(out["cpu_baseline"])
        if isinstance(cb.get("scipy"), dict):
            cb["scipy"] = {k: _r(cb["scipy"][k]) for k in ("value", "rel_inf_vs_gpu") if k in cb["scipy"]}
        cb["value"] = _r(cb["value"])
        out["cpu_baseline"] = cb
    mg = line.get("mg_apply")
    if isinstance(mg, dict) and "error" not in mg:
        out["mg_apply"] = {"value": _r(mg["value"]), "unit": mg["unit"], "ms_per_step": _r(mg["ms_per_step"]),
                           "inner": "mg:1/mg:1", "f_numerics": mg.get("f_numerics"), "launch": mg.get("launch"),
                           "setup_seconds": _r(mg.get("setup_seconds"), 3),
                           "levels": f"{mg['levels_F'][0]}^2..{mg['levels_F'][-1]}^2",
                           "roofline": _roof(mg.get("roofline"))}
        if isinstance(mg.get("roofline_stored_level1"), dict):
            s = mg["roofline_stored_level1"]
            out["mg_apply"]["roofline_stored_level1"] = {"kernel": s["kernel"].split(" (")[0], "frac": _r(s["frac"]),
                                                         "avg_launch_us": _r(s["avg_launch_us"])}
    elif mg is not None:
        out["mg_apply"] = mg
    if isinstance(line.get("host_buffer_matvec"), dict):
        out["host_buffer_matvec"] = {"value": _r(line["host_buffer_matvec"]["value"]), "unit": "applies/s",
                                     "note": "host ndarray in and out over PCIe per call"}
    sl = line.get("solve_level")
    if isinstance(sl, dict) and sl.get("runs") is not None:
        cols = ("n", "eta_n", "preconditioner", "iterations", "converged", "seconds", "apply_ms", "true_rel_residual")
        out["solve_level"] = {"tol": sl["tol"], "maxiter": sl["maxiter"], "problem": "solve.py:52-80, x0 = 0",
                              "f_numerics": sl.get("f_numerics"), "cols": list(cols),
                              "runs": [[_r(r.get(c)) for c in cols] for r in sl["runs"]]}
    tts = line.get("time_to_solution")
    if isinstance(tts, dict):
        out["time_to_solution"] = {k: {kk: _r(vv) for kk, vv in v.items() if vv is not None} for k, v in tts.items()}
    sp, rc = line.get("spmv_A"), line.get("roofline_csr_spmv")
    if isinstance(rc, dict):
        cal = rc.get("same_run_stream") or {}
        out["roofline_csr_spmv"] = {
            **_roof(rc),
            "back_to_back_us": _r(rc.get("back_to_back_us")), "frac_back_to_back": _r(rc.get("frac_back_to_back")),
            "sell_frac": _r(sp["sell_gbs"] / HBM_PEAK_GBS) if isinstance(sp, dict) and "sell_gbs" in sp else None,
            "same_run_stream": {"read_frac": _r(cal["read"]["frac_of_peak"]),
                                "spmv_shape_frac": _r(cal["spmv_shape"]["frac_of_peak"]),
                                "memory_clock": cal.get("memory_clock")} if cal else None,
            "frac_of_measured_stream": _r(rc.get("frac_of_measured_stream")),
            "timing": "HIP event pair around each of 20 launches"}
    contract = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")
    return {k: v for k, v in out.items() if v is not None or k in contract}


def _progress(rank, msg):
    """A progress line on stderr (rank 0): long sections (the N > 1 checks and solves) must not look hung; stdout keeps
    the one JSON line."""
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def timed_loop(fn, steps, warmup, world, dist, torch):
    """Seconds for `steps` calls of fn after `warmup` untimed ones, barrier + synchronize on both sides, max over
    ranks."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def partitioned_solver_section(args, n, rank, world, dist, torch, backend):
    """What the N > 1 line measures beyond the Chebyshev-4 headline apply: the configuration that SOLVES (FGMRES,
    solve.py:285, with one multigrid V-cycle per inner inverse -- the reference's pointer, solve.py:266 / 274) under the
    same row partition.
      mg_apply_partitioned: the mg:1 / mg:1 apply, applies/s in 1024^2-cell equivalents, eager (timed before any capture)
        and hipGraph-replayed (RCCL ranks);
      solve_distributed: FGMRES to 1e-8 on the manufactured problem (solve.py:52-80) over the ranks -- iterations,
        seconds (max over ranks) -- and, on rank 0, the one-GPU FGMRES of the same system: the residual histories must be
        identical bit for bit (reproducible inner products, bit-exact partitioned operator and preconditioner)."""
    import numpy as np
    import mp_block_preconditioners_amd as mp
    from mp_block_preconditioners_amd.distributed import DistributedMatrix, DistributedSchurPreconditioner
    scale = n * n / float(1024 * 1024)
    # the headline's numerics (--solve-numerics overrides): the partition's per-operator schedule starts its fast F
    # smoothing from the fast reciprocal diagonals as one GPU does (k_f_fast_init), so the residual histories are
    # comparable bit for bit in both numerics
    snum = args.solve_numerics or args.numerics
    mg1 = dict(inner_F=mp.InnerSolver("mg", 1, **MG_KW), inner_P=mp.InnerSolver("mg", 1, **MG_KW))
    out = {}
    t0 = time.perf_counter()
    M = DistributedSchurPreconditioner(n, args.xi, args.eta_n, args.eta_s, numerics=snum, **mg1)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0
    gen = torch.Generator(device="cuda").manual_seed(77 + rank)
    v = torch.randn(M.shape[0], dtype=torch.float64, device="cuda", generator=gen)
    o = torch.empty_like(v)
    _progress(rank, f"mg:1 partitioned preconditioner set up in {setup:.1f} s")
    dte = timed_loop(lambda: M.apply(v, o), args.steps, args.warmup, world, dist, torch)
    mg = {"inner": "mg:1 / mg:1", "unit": "applies/s (1024^2-cell equivalents)", "setup_seconds": setup,
          "eager_applies_per_s": args.steps / dte * scale, "f_numerics": snum,
          "level1": ("matrix-free, one launch over the rank's coarse rows (k_gal1 / k_gal1p)"
                     if snum == "fast" and n >= 72 and n % 2 == 0 else "stored Galerkin rows")}
    if backend == "nccl" and not args.eager_partitioned:
        try:
            g = M.capture(v, o)
            dtg = timed_loop(lambda: g.replay(), args.steps, args.warmup, world, dist, torch)
            mg.update({"applies_per_s": args.steps / dtg * scale, "launch": "hipgraph"})
            del g
        except Exception as e:
            mg.update({"applies_per_s": mg["eager_applies_per_s"], "launch": "eager",
                       "note": f"graph capture failed: {e}"})
    else:
        mg.update({"applies_per_s": mg["eager_applies_per_s"], "launch": "eager (host-staged gloo halo)"})
    M.close()
    del M
    torch.cuda.empty_cache()
    # FGMRES across the ranks (solve_distributed's steps, the fgmres call timed on its own)
    from mp_block_preconditioners_amd import _lib as L
    from mp_block_preconditioners_amd.distributed import RowPartition
    t0 = time.perf_counter()
    bp = mp.MultiphaseBlockPreconditioner(n, args.xi, args.eta_n, args.eta_s)
    own = torch.from_numpy(RowPartition(n, world, rank).owned_rows(5).astype(np.int32)).cuda()
    dA = DistributedMatrix(bp.assemble_rows(L.OP_A, own, c=1.0, d_u=-1.0), n, 5, owned_rows=True)
    del bp
    torch.cuda.empty_cache()
    Md = DistributedSchurPreconditioner(n, args.xi, args.eta_n, args.eta_s, numerics=snum, **mg1)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0
    _, b = mp.manufactured_problem(n, xi=args.xi, etan=args.eta_n, etas=args.eta_s)
    rows = dA.local_to_global_rows()
    bl = torch.from_numpy(np.ascontiguousarray(b[rows])).cuda()
    group = dist.group.WORLD
    hist = []
    dist.barrier()
    t0 = time.perf_counter()
    _progress(rank, f"distributed FGMRES set up in {setup:.1f} s")
    x, info = mp.fgmres(dA, bl, M=Md, tol=1e-8, maxiter=150, residuals=hist, group=group)
    _progress(rank, f"distributed FGMRES: {len(hist) - 1} iterations")
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    sd = {"inner": "mg:1 / mg:1", "tol": 1e-8, "maxiter": 150, "iterations": len(hist) - 1, "converged": info == 0,
          "seconds": el, "setup_seconds": setup, "rel_residual": hist[-1] / hist[0] if hist and hist[0] else None,
          "halo": Md.halo_impl, "preconditioner_comm_refs": (Md._rccl.comm_refs if Md._rccl is not None else 0),
          "f_numerics": snum}
    own_comm = None if Md._rccl is None or dA._rccl is None else bool(Md._rccl.comm != dA._rccl.comm)
    dA.close()
    Md.close()
    del dA, Md, x
    torch.cuda.empty_cache()
    same = torch.tensor([1], dtype=torch.int64, device="cuda")
    if rank == 0 and not args.no_check:
        t0 = time.perf_counter()
        bp = mp.MultiphaseBlockPreconditioner(n, args.xi, args.eta_n, args.eta_s)
        A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
        # the one-GPU default: level 1 matrix-free in one launch (k_gal1 / k_gal1p) as the partition runs it over each
        # rank's owned coarse rows, Gt_F_G's symmetric half on both sides (q13_mf: its default, spelled out)
        pc1 = mp.ApproxSchurPreconditioner(F, D, G, numerics=snum, **mg1, kernel_opts={"q13_mf": 0})
        h1 = []
        mp.fgmres(A, torch.from_numpy(b).cuda(), M=pc1, tol=1e-8, maxiter=150, residuals=h1)
        same[0] = 1 if np.array_equal(np.asarray(h1), np.asarray(hist)) else 0
        sd["single_gpu_iterations"] = len(h1) - 1
        sd["single_gpu_check_seconds"] = time.perf_counter() - t0
        del pc1, A, F, D, G, bp
        torch.cuda.empty_cache()
    dist.all_reduce(same, op=dist.ReduceOp.MIN)
    if not args.no_check:
        sd["bit_exact_vs_single_gpu"] = bool(same.item())
        sd["check"] = ("the residual history (every iteration's ||r||) equals the one-GPU FGMRES's bit for bit (the "
                       "one-GPU default kernel choices)")
    if own_comm is not None:   # A u's eager side-stream exchanges never share a communicator with graph-replayed ones
        sd["operator_has_its_own_communicator"] = own_comm
    return {"mg_apply_partitioned": mg, "solve_distributed": sd}


def launch_ranks(n_ranks):
    """Run this command line as n_ranks torch.distributed.run ranks (127.0.0.1 rendezvous) in a child process
    and return its exit status.  Called before torch is imported: the parent never touches the GPU."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n_ranks}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def single_gpu_check(dpc, n, args, iF, iP, rank, dist, torch):
    """The partitioned apply of a global random vector against the one-GPU apply (every rank, its rows)."""
    import numpy as np
    import mp_block_preconditioners_amd as mp
    t0 = time.perf_counter()
    bp = mp.MultiphaseBlockPreconditioner(n, args.xi, args.eta_n, args.eta_s)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    # (the one-GPU default apply: the partition reads Gt_F_G's symmetric half over its row block as one GPU does)
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP, layout=args.layout, f_mode=args.f_mode,
                                      pg_mode=args.pg_mode, numerics=args.numerics, kernel_opts={"q13_mf": 0})
    del F, D, G
    vg = torch.from_numpy(np.random.default_rng(2048).standard_normal(pc.shape[0])).cuda()
    gids = torch.from_numpy(dpc.local_to_global_rows()).cuda()
    ref = pc.apply(vg)[gids]
    got = dpc.apply(vg[gids].contiguous())
    torch.cuda.synchronize()
    same = torch.tensor([1 if torch.equal(got, ref) else 0], dtype=torch.int64, device="cuda")
    csum = got.view(torch.int64).sum().reshape(1)
    dist.all_reduce(same, op=dist.ReduceOp.MIN)
    dist.all_reduce(csum, op=dist.ReduceOp.SUM)
    ok = bool(same.item())
    del pc
    torch.cuda.empty_cache()
    return {"bit_exact": ok, "output_bits_sum_mod_2^64": int(csum.item()) & (2 ** 64 - 1),
            "note": "every rank's rows of the partitioned apply vs the single-GPU apply of the same global "
                    f"vector (numpy seed 2048), built on each rank's GPU; {time.perf_counter() - t0:.1f} s"}


EVENT_NOTE = ("hipEvents with a device-scope release (hipEventReleaseToDevice, mpbp_event_create_scoped): recording "
              "one does not write the L2 back, so the kernel between a pair runs as inside the captured apply; "
              "MPBP_EVENT_SCOPE=system: hipEventDefault") if os.environ.get("MPBP_EVENT_SCOPE", "device") != "system" \
    else "hipEventDefault (system-scope release after every recorded event; MPBP_EVENT_SCOPE=system)"


def spmv_bench(A, gen, reps=20, replays=10, warm_replays=5):
    """The plain operator matvec b = A u (apply.py:72) in both layouts, HIP-event timed.

    The kernel's launch duration (`*_us`, what the roofline divides by and what rocprof's kernel trace
    reports) is the mean over `reps` launches of a HIP event pair recorded around each launch.  Beside it:
    `reps` back-to-back launches captured into one hipGraph and replayed `replays` times between two events
    (`*_us_graph`: per launch including the drain / dispatch gap between dependent kernels), and the eager
    loop (`*_us_eager`)."""
    import torch
    from mp_block_preconditioners_amd.solve import DeviceEvent
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    x = torch.randn(A.shape[1], dtype=torch.float64, device="cuda", generator=gen)
    y = torch.empty(A.shape[0], dtype=torch.float64, device="cuda")
    res = {"nnz": A.nnz, "timing": f"mean of HIP event pairs around each of {reps} launches (after "
                                   f"{replays} graph replays of {reps} back-to-back launches, `*_us_graph`)"}
    AS = A.to_sell()
    # CSR algorithmic bytes: 12 B per entry (value + column) + x and y (8 B per row / column) + the row structure the
    # kernel reads: with the row blocks' wave table (default) 32 B per block, and row_ptr (4 B per row) + the block's
    # row range (8 B) only for waves the table does not flag uniform; without it row_ptr for every row
    tb = A.blocks.table
    if tb is not None:
        import numpy as np
        t = tb.cpu().numpy().reshape(-1, 8).astype(np.int64)
        nonuni = 0
        for w in range(4):
            rows_w = np.clip(t[:, 1] - (t[:, 0] + 64 * w), 0, 64)
            nonuni += int(rows_w[((t[:, 7] >> (8 * w)) & 255) == 0].sum())
        struct_bytes = A.blocks.count * 32 + (nonuni * 4 + A.blocks.count * 8 if nonuni else 0)
    else:
        struct_bytes = (A.shape[0] + 1) * 4 + A.blocks.count * 8
    csr_bytes = A.nnz * 12 + (A.shape[0] + A.shape[1]) * 8 + struct_bytes
    for name, M, nbytes in (
            ("csr", A, csr_bytes),              # per-wave chunked kernel (k_csr_wave)
            ("sell", AS, A.nnz * 12 + A.shape[0] + (A.shape[0] + A.shape[1]) * 8 + AS.nslices * 16)):
        for _ in range(3):
            M.matvec(x, out=y)
        ev[0].record()
        for _ in range(reps):
            M.matvec(x, out=y)
        ev[1].record()
        torch.cuda.synchronize()
        s_eager = ev[0].elapsed_time(ev[1]) / 1e3 / reps
        s = s_eager
        try:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                M.matvec(x, out=y)
            torch.cuda.current_stream().wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(reps):
                    M.matvec(x, out=y)
            for _ in range(warm_replays):   # the clock settles under the sustained stream before timing
                g.replay()
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(replays):
                g.replay()
            ev[1].record()
            torch.cuda.synchronize()
            s = ev[0].elapsed_time(ev[1]) / 1e3 / (reps * replays)
            del g
        except Exception as e:   # eager number only, and say why
            res[f"{name}_graph_note"] = f"graph capture failed: {e}"
        pairs = [(DeviceEvent(), DeviceEvent()) for _ in range(reps)]
        for a, b in pairs:   # right after the graph replays: the clock is settled
            a.record()
            M.matvec(x, out=y)
            b.record()
        torch.cuda.synchronize()
        s_launch = sum(a.elapsed_ms(b) for a, b in pairs) / 1e3 / reps
        res.update({f"{name}_gbs": nbytes / s_launch / 1e9, f"{name}_us": s_launch * 1e6, f"{name}_bytes": nbytes,
                    f"{name}_us_graph": s * 1e6, f"{name}_gbs_graph": nbytes / s / 1e9,
                    f"{name}_us_eager": s_eager * 1e6})
    res["calibration"] = hbm_calibration(csr_bytes, reps)
    return res


def hbm_calibration(nbytes, reps=20):
    """Same-run, same-size HBM reference rates for the CSR SpMV roofline (mpbp_hbm_stream, timed like the SpMV: a HIP
    event pair around each of `reps` launches after 30 warm launches): `read` streams nbytes once in order; `spmv_shape`
    moves the SpMV's own stream shape without its x gathers (per 64-row wave 9 KiB read in order + 512 B written), about
    the same byte count.  frac_of_measured_stream = the SpMV's GB/s over spmv_shape's: what separates the kernel from
    the box.  Plus the memory clock rocm-smi reports (None where it cannot be read)."""
    import torch
    from mp_block_preconditioners_amd._lib import check, lib, ptr, stream_handle
    from mp_block_preconditioners_amd.solve import DeviceEvent
    src = torch.empty(nbytes // 8 + 2048, dtype=torch.float64, device="cuda")
    src.fill_(0.5)
    nw = nbytes // (576 * 16)
    dst = torch.empty(max(256, nw * 64), dtype=torch.float64, device="cuda")
    out = {}
    for name, mode, moved in (("read", 0, nbytes // 16 * 16), ("spmv_shape", 1, nw * (576 * 16 + 512))):
        def launch():
            check(lib().mpbp_hbm_stream(ptr(src), nbytes, mode, ptr(dst), stream_handle()))
        for _ in range(30):
            launch()
        pairs = [(DeviceEvent(), DeviceEvent()) for _ in range(reps)]
        for a, b in pairs:
            a.record()
            launch()
            b.record()
        torch.cuda.synchronize()
        us = sum(a.elapsed_ms(b) for a, b in pairs) * 1e3 / reps
        out[name] = {"bytes": moved, "avg_launch_us": us, "gbs": moved / us / 1e3, "frac_of_peak": moved / us / 1e3 / HBM_PEAK_GBS}
    del src, dst
    torch.cuda.empty_cache()
    out["memory_clock"] = memory_clock()
    return out


def memory_clock():
    """The current memory clock as rocm-smi prints it (MCLK), or None."""
    import re
    import subprocess
    try:
        txt = subprocess.run(["rocm-smi", "--showclocks"], capture_output=True, text=True, timeout=20).stdout
    except (OSError, subprocess.SubprocessError):
        return None
    for line in txt.splitlines():
        if "mclk" in line.lower():
            m = re.search(r"\(([0-9.]+\s*[MG]hz)\)", line, re.I)
            return m.group(1) if m else line.strip()
    return None


def mg_apply_bench(F, D, G, steps, warmup, gen, reps=20, numerics="exact"):
    """The apply with one multigrid V-cycle per inner inverse (mg:1 / mg:1: the configuration that converges FGMRES in
    solve_level, solve.py:266 / 274's pointer), hipGraph-replayed as the headline apply, and the roofline of its
    dominant kernel family: the level-1 F Galerkin operator's Chebyshev sweep (8 launches per apply at 1024^2) on the
    layout the apply uses (stencil values, k_svl<EpiCheb>; else SELL-64), HIP events around each of `reps` launches
    of that kernel on the level's own buffers."""
    import ctypes
    import torch
    import mp_block_preconditioners_amd as mp
    from mp_block_preconditioners_amd._lib import check, lib, ptr, stream_handle
    from mp_block_preconditioners_amd.solve import DeviceEvent
    t0 = time.perf_counter()
    pc = mp.ApproxSchurPreconditioner(F, D, G, inner_F=mp.InnerSolver("mg", 1, **MG_KW),
                                      inner_P=mp.InnerSolver("mg", 1, **MG_KW),
                                      numerics=numerics)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    v = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda", generator=gen)
    out = torch.empty_like(v)
    g = pc.capture(v, out)
    for _ in range(warmup):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    del g
    mg = pc.mg_F
    S, M1, w, dg, V = mg.sells[0][1], mg.ops[1], mg.work[1], mg.diags[1], mg.svls[1]
    c1, c2 = (ctypes.c_double * 2)(), (ctypes.c_double * 2)()
    check(lib().mpbp_cheb_coeffs(mg.bounds[1][0], mg.bounds[1][1], 2, c1, c2))
    x, xo, d, b = w[0], w[1], w[3], w[4]
    x.normal_(generator=gen)
    b.normal_(generator=gen)
    d.zero_()
    def sweep():
        if V is not None:
            check(lib().mpbp_svl_cheb_step(ctypes.byref(V.cstruct()), ctypes.byref(M1.cstruct()), ptr(x), ptr(b),
                                           ptr(dg), c1[1], c2[1], ptr(d), None, ptr(xo), stream_handle()))
        else:
            check(lib().mpbp_sell_cheb_step(ctypes.byref(S.cstruct()), ptr(x), ptr(b), ptr(dg), c1[1], c2[1], ptr(d),
                                            None, ptr(xo), stream_handle()))
    for _ in range(3):
        sweep()
    pairs = [(DeviceEvent(), DeviceEvent()) for _ in range(reps)]
    for a, e in pairs:
        a.record()
        sweep()
        e.record()
    torch.cuda.synchronize()
    us = sum(a.elapsed_ms(e) for a, e in pairs) * 1e3 / reps
    rows = M1.shape[0]
    stored = {"kernel": None, "avg_launch_us": us}
    # per row x (gathered, counted once), b, diag, d read, d written, x_out (8 B each); the matrix: stencil values 8 B
    # per entry (edge rows: their CSR entries, 12 B, + 4 B row_ptr), or SELL 12 B per entry + 1 B row length + 16 B
    # per slice descriptor
    if V is not None:
        ne, K = int(V.edge_rows.numel()), V.slots
        nbytes = (rows - ne) * K * 8 + ne * (K * 12 + 4) + rows * 6 * 8
        kname = f"k_svl<EpiCheb> (level-1 F Galerkin operator, {rows} rows x {K} entries, stencil values)"
    else:
        nbytes = M1.nnz * 12 + rows * (1 + 6 * 8) + S.nslices * 16
        kname = f"k_sell_rows<EpiCheb> (level-1 F Galerkin operator, {rows} rows x {M1.nnz / rows:.0f} entries, SELL-64)"
    stored = {"bound": "hbm", "achieved": nbytes / us / 1e3, "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "frac": nbytes / us / 1e3 / HBM_PEAK_GBS, "kernel": kname, "bytes_per_launch": nbytes,
              "avg_launch_us": us, "launches_per_apply": 8,
              "timing": f"mean of HIP event pairs around each of {reps} launches on the level's buffers",
              "events": EVENT_NOTE}
    res = {"value": 1.0 / dt, "unit": "applies/s", "ms_per_step": dt * 1e3, "inner_F": "mg:1", "inner_P": "mg:1",
           "f_numerics": numerics,
           "setup_seconds": setup_s, "launch": "hipgraph",
           "levels_F": mg.sizes, "levels_P": pc.mg_P.sizes, "roofline": stored}
    if numerics == "fast":
        # the tolerance mode never runs that sweep: level 1 of F is R0 (F (P0 x)) in one k_gal1 launch (3 Chebyshev
        # sweeps + 1 residual per apply).  Time it through mpbp_mg_level1_apply (residual epilogue) on the plan itself.
        n = int(pc._plan.f_prm.n)
        r1 = 4 * (n // 2) ** 2
        xr, zr, yr = (torch.randn(r1, dtype=torch.float64, device="cuda", generator=gen) for _ in range(3))

        def gal1():
            check(lib().mpbp_mg_level1_apply(ctypes.byref(pc._plan), 0, 2, ptr(xr), ptr(zr), ptr(yr),
                                             stream_handle()))
        for _ in range(3):
            gal1()
        pairs = [(DeviceEvent(), DeviceEvent()) for _ in range(reps)]
        for a, e in pairs:
            a.record()
            gal1()
            e.record()
        torch.cuda.synchronize()
        ug = sum(a.elapsed_ms(e) for a, e in pairs) * 1e3 / reps
        # algorithmic bytes: coarse x, the residual's rhs z and output y (8 B per level-1 row each) and the fine thn
        # tables the F rows read (cell, u-face, v-face: 3 x 8 B per fine cell); t0 = P0 x and t1 = F t0 live in LDS
        gb = r1 * 3 * 8 + 3 * n * n * 8
        res["roofline_stored_level1"] = stored
        res["roofline"] = {
            "bound": "hbm", "achieved": gb / ug / 1e3, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gb / ug / 1e3 / HBM_PEAK_GBS,
            "kernel": f"k_gal1<EpiResid, MAC> (level-1 F operator R0 (F (P0 x)) matrix-free, {r1} coarse rows, "
                      f"one launch)", "bytes_per_launch": gb, "avg_launch_us": ug, "launches_per_apply": 4,
            "timing": f"mean of HIP event pairs around each of {reps} mpbp_mg_level1_apply launches",
            "events": EVENT_NOTE,
            "note": "the apply runs this kernel 3x with the Chebyshev epilogue and 1x with the residual one; its HBM "
                    "bytes are small beside its work (P0, the 4-field F rows and R0 recomputed on a 64 x 8 fine "
                    "block + halo per workgroup): issue-bound, not HBM-bound -- frac says how far from the HBM "
                    "floor the kernel sits. roofline_stored_level1 is the stored-matrix sweep the exact mode streams"}
    return res


SOLVE_CASES = (   # (n, eta_n, eta_s, preconditioners): BASELINE configs[1] / configs[3] at 256^2, configs[2] / [3] at 1024^2
    (256, 100.0, 1.0, ("none", "chebyshev:4", "mg:1")),
    (256, 1e4, 1.0, ("none", "chebyshev:4", "mg:1", "mg:2/mg:1")),
    (1024, 100.0, 1.0, ("chebyshev:4", "mg:1", "mg:2/mg:1", "mg:4/mg:1", "mg:8/mg:1")),
    (1024, 1e4, 1.0, ("chebyshev:4", "mg:1", "mg:2/mg:1", "mg:4/mg:1", "mg:8/mg:1")),
)


def inner_pair(mp, name):
    """'kind:k' (both inner inverses) or 'kindF:kF/kindP:kP' -> (InnerSolver for F, InnerSolver for Gt_G); a suffix
    '@pre,post' sets the multigrid smoothing sweeps (default V(2,2))."""
    name, _, smooth = name.partition("@")
    mgkw = {}
    if smooth:
        pre, _, post = smooth.partition(",")
        mgkw = dict(pre=int(pre), post=int(post or pre))
    f, _, p = name.partition("/")

    def mk(s):
        kind, _, k = s.partition(":")
        return mp.InnerSolver(kind, int(k or 4), **({**MG_KW, **mgkw} if kind == "mg" else {}))
    return mk(f), mk(p or f)


def solve_level(args, cases=SOLVE_CASES, tol=1e-8, maxiter=150, reps=10):
    """What the applies/s headline buys: FGMRES (tol 1e-8, maxiter 150, x0 = 0, solve.py:285) on the reference's
    manufactured problem (solve.py:52-80) with the approximate Schur preconditioner and different inner solves:
    iterations, time to tolerance (the fgmres call, replaying the apply's hipGraph; preconditioner set-up and the
    graph capture reported apart), the velocity error, and the preconditioner's own apply time (the graph replayed
    `reps` times)."""
    import numpy as np
    import torch
    import mp_block_preconditioners_amd as mp
    out = []
    for n, eta_n, eta_s, precs in cases:
        bp = mp.MultiphaseBlockPreconditioner(n, args.xi, eta_n, eta_s)
        A, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
        u, b = mp.manufactured_problem(n, xi=args.xi, etan=eta_n, etas=eta_s)
        bd = torch.from_numpy(b).cuda()
        nb = float(torch.linalg.vector_norm(bd))
        for name in precs:
            t0 = time.perf_counter()
            M = None
            apply_ms = None
            if name != "none":
                iF, iP = inner_pair(mp, name)
                M = mp.ApproxSchurPreconditioner(F, D, G, inner_F=iF, inner_P=iP, numerics=args.numerics)
            torch.cuda.synchronize()
            setup = time.perf_counter() - t0
            capture_s = None
            if M is not None:
                v = torch.randn(M.shape[0], dtype=torch.float64, device="cuda")
                o = torch.empty_like(v)
                t0 = time.perf_counter()
                g = M.capture(v, o)
                torch.cuda.synchronize()
                capture_s = time.perf_counter() - t0
                g.replay()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    g.replay()
                torch.cuda.synchronize()
                apply_ms = (time.perf_counter() - t0) / reps * 1e3
                M._fgmres_graph = (v, o, g)   # the solve replays this capture (fgmres reuses a graph kept on M)
                del g, v, o
            hist = []
            t0 = time.perf_counter()
            x, info = mp.fgmres(A, bd, M=M, tol=tol, maxiter=maxiter, residuals=hist)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            res = float(torch.linalg.vector_norm(bd - A.matvec(x))) / nb
            err = float(np.max(np.abs(x.cpu().numpy()[: 4 * n * n] - u[: 4 * n * n])))
            out.append({"n": n, "eta_n": eta_n, "eta_s": eta_s, "preconditioner": name, "iterations": len(hist) - 1,
                        "converged": info == 0, "seconds": el, "setup_seconds": setup, "capture_seconds": capture_s,
                        "apply_ms": apply_ms,
                        "true_rel_residual": res, "velocity_max_error": err})
            del M, x
            torch.cuda.empty_cache()
        del A, F, D, G, bp
        torch.cuda.empty_cache()
    return {"tol": tol, "maxiter": maxiter, "problem": "manufactured solution of solve.py:52-80, x0 = 0",
            "f_numerics": args.numerics,
            "inner": "chebyshev:K = K Chebyshev-Jacobi sweeps; mg:K = K multigrid V-cycles (V(2,2), Chebyshev "
                     "smoothing, Galerkin levels down to 16^2, its dense inverse there; '@a,b': V(a,b)); 'F/P' names "
                     "the two inner inverses separately",
            "runs": out}


def cpu_baseline(pc, v, seconds, kf, sf, kp, spp, numerics="exact"):
    """The oracle's apply (sequential C, one core) on the same matrices, bounded sample; the GPU apply of the same
    vector is checked against the timed oracle output: bit for bit (exact numerics) or within north_star's 1e-12
    relative inf-norm (fast numerics)."""
    import numpy as np
    from oracle.schur_oracle import Inner, approx_schur_apply
    Fh, Dh, Gh = pc.F.to_scipy(), pc.D.to_scipy(), pc.G.to_scipy()
    GtGh, GtFGh = pc.GtG.to_scipy(), pc.GtFG.to_scipy()
    iF = Inner(kf, sf, pc.inner_F.lmin or 0.0, pc.inner_F.lmax or 0.0)
    iP = Inner(kp, spp, pc.inner_P.lmin or 0.0, pc.inner_P.lmax or 0.0)
    dF, dP = pc.diag_F.cpu().numpy(), pc.diag_P.cpu().numpy()
    vh = v.cpu().numpy()
    done = 0
    t0 = time.perf_counter()
    while True:
        ref = approx_schur_apply(Fh, Dh, Gh, GtGh, GtFGh, vh, iF, iP, diag_F=dF, diag_P=dP)
        done += 1
        if time.perf_counter() - t0 >= seconds:
            break
    el = time.perf_counter() - t0
    # the GPU apply of the same vector must be bit-identical to the timed oracle output
    gpu = pc.apply(v).cpu().numpy()
    same = bool(np.array_equal(gpu.view(np.uint64), ref.view(np.uint64)))
    orel = float(np.max(np.abs(gpu - ref)) / np.max(np.abs(ref)))
    # the reference's own CPU form of the same apply: scipy.sparse `@` products + numpy vectors
    from oracle.schur_oracle import approx_schur_apply_scipy
    sdone = 0
    t0 = time.perf_counter()
    while True:
        sref = approx_schur_apply_scipy(Fh, Dh, Gh, GtGh, GtFGh, vh, iF, iP, dF, dP)
        sdone += 1
        if time.perf_counter() - t0 >= seconds:
            break
    sel = time.perf_counter() - t0
    srel = float(np.max(np.abs(sref - gpu)) / np.max(np.abs(gpu)))
    return {"value": done / el, "unit": "applies/s", "cores": 1, "kind": "port",
            "sample": f"{done} full applies of the same {pc.shape[0]}-unknown system in {el:.1f} s "
                      f"(oracle/csr_oracle.c, 1 thread)", "bit_exact_vs_gpu": same,
            "rel_inf_vs_gpu": orel, "gpu_numerics": numerics,
            "parity": ("bit-exact" if same else "FAILED") if numerics == "exact" else
                      ("within 1e-12 relative inf-norm" if orel <= 1e-12 else "FAILED (above 1e-12)"),
            "scipy": {"value": sdone / sel, "unit": "applies/s", "cores": 1,
                      "sample": f"{sdone} applies composed from scipy.sparse CSR products (the reference's "
                                f"CPU form, solve.py:257-277) in {sel:.1f} s, 1 thread",
                      "rel_inf_vs_gpu": srel}}


if __name__ == "__main__":
    sys.exit(main() or 0)
