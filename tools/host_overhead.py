"""Host-side enqueue time of one apply versus its GPU time (is the eager partitioned apply host-bound?).

    python tools/host_overhead.py [--self-halo] [--grid 1024]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=1024)
    ap.add_argument("--self-halo", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    import mp_block_preconditioners_amd as mpb
    torch.cuda.set_device(0)
    if args.self_halo:
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:29581", rank=0, world_size=1)
        from mp_block_preconditioners_amd.distributed import DistributedSchurPreconditioner
        pc = DistributedSchurPreconditioner(args.grid, 1.0, 100.0, 1.0, halo="rccl", self_halo=True)
    else:
        bp = mpb.MultiphaseBlockPreconditioner(args.grid, 1.0, 100.0, 1.0)
        _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
        pc = mpb.ApproxSchurPreconditioner(F, D, G)
    v = torch.randn(pc.shape[0], dtype=torch.float64, device="cuda")
    out = torch.empty_like(v)
    for _ in range(3):
        pc.apply(v, out)
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(args.reps):
        t = time.perf_counter()
        pc.apply(v, out)
        host.append(time.perf_counter() - t)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"grid {args.grid} self_halo {args.self_halo}: host enqueue {1e6 * sum(host) / len(host):.0f} us/apply "
          f"(min {1e6 * min(host):.0f}), wall {1e6 * t_all / args.reps:.0f} us/apply, "
          f"enqueue loop {1e6 * t_enq / args.reps:.0f} us/apply", flush=True)
    if args.self_halo:
        pc.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
