"""Probe: hipGraph capture of the row-partitioned apply with the RCCL halo (one GPU, periodic self-exchange).

    timeout -k 10 120 python tools/capture_probe.py 256 1024

For every grid size: eager apply, capture (thread-local error mode), replay, bit-compare, and time
eager vs replayed applies.  Prints one line per step so a hang names the step it happened in.
"""
import gc
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    sizes = [int(a) for a in sys.argv[1:]] or [256, 1024]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{29500 + os.getpid() % 1000}", rank=0,
                            world_size=1, device_id=torch.device("cuda", 0))
    import mp_block_preconditioners_amd as mp
    from mp_block_preconditioners_amd.distributed import DistributedSchurPreconditioner
    for n in sizes:
        iF, iP = mp.InnerSolver("chebyshev", 4), mp.InnerSolver("chebyshev", 4)
        print(f"n={n} setup", flush=True)
        dpc = DistributedSchurPreconditioner(n, 1.0, 100.0, 1.0, inner_F=iF, inner_P=iP, self_halo=True)
        print(f"n={n} setup done", flush=True)
        v = torch.randn(dpc.shape[0], dtype=torch.float64, device="cuda")
        ref = dpc.apply(v).clone()
        torch.cuda.synchronize()
        print(f"n={n} eager ok (ca={dpc.ca}, h={dpc.h_u}/{dpc.h_p})", flush=True)
        out = torch.zeros_like(v)
        g = dpc.capture(v, out)
        torch.cuda.synchronize()
        print(f"n={n} captured", flush=True)
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        print(f"n={n} replay bit-exact: {torch.equal(out, ref)}", flush=True)
        for name, fn in (("eager", lambda: dpc.apply(v, out)), ("graph", g.replay)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
            print(f"n={n} {name}: {20 / (time.perf_counter() - t0):.0f} applies/s", flush=True)
        del g
        gc.collect()
        torch.cuda.synchronize()
        print(f"n={n} graph destroyed", flush=True)
        dpc.close()
        print(f"n={n} halo communicator destroyed", flush=True)
    dist.destroy_process_group()
    print("process group destroyed", flush=True)


if __name__ == "__main__":
    main()
