"""A/B timing of the CSR SpMV kernels on the 1024^2 operator A (apply.py:72), for experiment builds.

    MPBP_LIB=.../libmpbp_<variant>.so python tools/spmv_ab.py [--n 1024] [--reps 50]

Prints one JSON line: per CSR kernel kind the mean HIP-event time and algorithmic GB/s, the SELL time,
and whether each CSR result is bit-identical to the SELL result (same CSR-order sums).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import torch
    import mp_block_preconditioners_amd as mp
    bp = mp.MultiphaseBlockPreconditioner(args.n, 1.0, 100.0, 1.0, device="cuda:0")
    A = bp.get_big_A_matrix(c=1.0, d_u=-1.0)[0]
    gen = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(A.shape[1], dtype=torch.float64, device="cuda", generator=gen)
    y = torch.empty(A.shape[0], dtype=torch.float64, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    AS = A.to_sell()
    ref = AS.matvec(x).clone()
    nbytes = A.nnz * 12 + (A.shape[0] + 1) * 4 + (A.shape[0] + A.shape[1]) * 8 + A.blocks.count * 8
    res = {"n": args.n, "nnz": A.nnz, "lib": os.environ.get("MPBP_LIB", "default")}
    flat = A.plan_blocks(groups=1)   # blocks in plain row order (no per-field interleave)
    from mp_block_preconditioners_amd._lib import check, lib
    runs = [("csr_wave", A, None, "seq"), ("csr_wave_notable", A, None, "notable"), ("csr_seg", A, None, "seg"),
            ("csr_wave_roworder", A, flat, "seq"), ("sell", AS, None, None)]
    for name, M, blk, order in runs:
        kw = {"blocks": blk} if blk is not None else {}
        check(lib().mpbp_set_csr_table(0 if order == "notable" else 1))
        if order == "seg":
            kw["order"] = "seg"
        for _ in range(5):
            M.matvec(x, out=y, **kw)
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(args.reps):
            M.matvec(x, out=y, **kw)
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1e3 / args.reps
        res[name] = {"us": round(us, 2), "gbs": round(nbytes / us / 1e3, 1),
                     "bit_exact_vs_sell": bool(torch.equal(y.view(torch.int64), ref.view(torch.int64))),
                     "rel_inf_vs_sell": float((y - ref).abs().max() / ref.abs().max())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
