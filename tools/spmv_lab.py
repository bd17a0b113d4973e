"""CSR SpMV lab on the 1024^2 operator A (apply.py:72): the product kernel, its staging / cache-policy alternatives
(tools/spmv_lab.hip) and same-run HBM calibrations, all interleaved in one process on one box.

    python tools/spmv_lab.py [--build] [--n 1024] [--rounds 3] [--reps 20]

Prints one JSON line per round and a summary line: per variant the mean per-launch HIP-event time (warm: after
back-to-back launches; cold: after a 512 MiB write that evicts the Infinity Cache), the back-to-back time, and
GB/s of the SpMV's algorithmic bytes (the bench's byte count).  Variants' results are checked bit-identical to the
product kernel's.
"""
import argparse
import ctypes

import numpy as np
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LAB = os.path.join(ROOT, "tools", "lab", "libspmv_lab.so")


def build():
    os.makedirs(os.path.dirname(LAB), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-ffp-contract=off", os.path.join(ROOT, "tools", "spmv_lab.hip"), "-o", LAB])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    if args.build:
        build()
        return
    import torch
    import mp_block_preconditioners_amd as mp
    from mp_block_preconditioners_amd._lib import stream_handle
    from mp_block_preconditioners_amd.solve import DeviceEvent
    L = ctypes.CDLL(LAB)
    P = ctypes.c_void_p
    L.lab_read.argtypes = [P, ctypes.c_int64, ctypes.c_int, P, P]
    L.lab_readwrite.argtypes = [P, ctypes.c_int64, ctypes.c_int, P, P]
    L.lab_fill.argtypes = [P, ctypes.c_int64, ctypes.c_double, P]
    L.lab_csr.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_int32, P, ctypes.c_int, P, P]

    bp = mp.MultiphaseBlockPreconditioner(args.n, 1.0, 100.0, 1.0, device="cuda:0")
    A = bp.get_big_A_matrix(c=1.0, d_u=-1.0)[0]
    gen = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(A.shape[1], dtype=torch.float64, device="cuda", generator=gen)
    y = torch.empty(A.shape[0], dtype=torch.float64, device="cuda")
    blk = A.blocks
    tb = blk.table
    assert tb is not None
    nbytes = A.nnz * 12 + (A.shape[0] + A.shape[1]) * 8 + blk.count * 32
    ref = A.matvec(x).clone()
    buf = torch.empty(nbytes // 8 + 1024, dtype=torch.float64, device="cuda")
    buf.normal_(generator=gen)
    nwaves = A.shape[0] // 64
    rw_bytes = nwaves * (9 * 1024 + 512)
    flush = torch.empty(512 * 1024 * 1024 // 8, dtype=torch.float64, device="cuda")
    sink = torch.zeros(256, dtype=torch.float64, device="cuda")
    ybuf = torch.empty(nwaves * 64, dtype=torch.float64, device="cuda")

    def sh():
        return stream_handle()

    def lab_csr(mode, nt, table=None):
        t = tb if table is None else table
        return lambda: L.lab_csr(mode, nt, P(A.val.data_ptr()), P(A.col_idx.data_ptr()), P(x.data_ptr()),
                                 A.shape[1], P(t.data_ptr()), blk.count, P(y.data_ptr()), sh())

    # block orders: the product's (fields interleaved block by block across the 5 stacked fields), plain row order,
    # and the fields interleaved in chunks of q consecutive blocks (fewer concurrent streams, x gathers still near)
    from mp_block_preconditioners_amd.csr import RowBlockList
    flat = A.plan_blocks(groups=1)
    fp = flat.pairs.cpu().numpy().reshape(-1, 2)
    nf = 5
    per = fp.shape[0] // nf
    tables = {"roworder": flat.table}
    for q in (4, 16):
        order = []
        for c0 in range(0, per, q):
            for f in range(nf):
                order.extend(range(f * per + c0, f * per + min(c0 + q, per)))
        order.extend(range(nf * per, fp.shape[0]))
        pq = np.ascontiguousarray(fp[np.asarray(order)].reshape(-1))
        tables[f"chunk{q}"] = RowBlockList(torch.from_numpy(pq).cuda(), A.row_ptr_host, pq).table

    # placement probes: the same product kernel with x / y in buffers allocated at other times (after 1.3 GB of other
    # allocations, and behind a 2 GiB spacer) -- does where x and y live change the rate (Infinity-Cache residency)?
    x_late = x.clone()
    spacer = torch.empty(2 * 1024 ** 3 // 8, dtype=torch.float64, device="cuda")
    x_far = torch.empty_like(x)
    x_far.copy_(x)
    y_late = torch.empty_like(y)

    variants = {
        "product_k_csr_wave": (lambda: A.matvec(x, out=y), nbytes, True),
        "product_x_late": (lambda: A.matvec(x_late, out=y), nbytes, True),
        "product_x_far": (lambda: A.matvec(x_far, out=y), nbytes, True),
        "product_y_late": (lambda: A.matvec(x, out=y_late), nbytes, False),
        "lab_reg_nt": (lab_csr(0, 1), nbytes, True),
        "lab_reg_default": (lab_csr(0, 0), nbytes, True),
        "lab_glds_nt": (lab_csr(1, 1), nbytes, True),
        "lab_glds_default": (lab_csr(1, 0), nbytes, True),
        "lab_glds_nt_noswizzle": (lab_csr(2, 1), nbytes, True),
        "lab_glds_aux3": (lab_csr(3, 1), nbytes, True),
        "lab_glds_aux1": (lab_csr(4, 1), nbytes, True),
        "lab_glds_roworder": (lab_csr(1, 1, tables["roworder"]), nbytes, True),
        "lab_glds_chunk4": (lab_csr(1, 1, tables["chunk4"]), nbytes, True),
        "lab_glds_chunk16": (lab_csr(1, 1, tables["chunk16"]), nbytes, True),
        "read_stream_nt": (lambda: L.lab_read(P(buf.data_ptr()), nbytes, 1, P(sink.data_ptr()), sh()), nbytes, False),
        "read_stream_default": (lambda: L.lab_read(P(buf.data_ptr()), nbytes, 0, P(sink.data_ptr()), sh()), nbytes,
                                False),
        "readwrite_nt": (lambda: L.lab_readwrite(P(buf.data_ptr()), nwaves, 1, P(ybuf.data_ptr()), sh()), rw_bytes,
                         False),
    }

    def do_flush():
        L.lab_fill(P(flush.data_ptr()), flush.numel(), 1.0, sh())

    ev = [DeviceEvent() for _ in range(2)]
    allres = {k: {"warm_us": [], "cold_us": [], "b2b_us": []} for k in variants}
    exact = {}
    for rnd in range(args.rounds):
        line = {"round": rnd}
        for name, (fn, nb, is_spmv) in variants.items():
            for _ in range(30):
                fn()
            torch.cuda.synchronize()
            pairs = [(DeviceEvent(), DeviceEvent()) for _ in range(args.reps)]
            for a, b in pairs:
                a.record()
                fn()
                b.record()
            torch.cuda.synchronize()
            warm = sum(a.elapsed_ms(b) for a, b in pairs) * 1e3 / args.reps
            ev[0].record()
            for _ in range(50):
                fn()
            ev[1].record()
            torch.cuda.synchronize()
            b2b = ev[0].elapsed_ms(ev[1]) * 1e3 / 50
            for a, b in pairs:
                do_flush()
                a.record()
                fn()
                b.record()
            torch.cuda.synchronize()
            cold = sum(a.elapsed_ms(b) for a, b in pairs) * 1e3 / args.reps
            if is_spmv:
                exact[name] = bool(torch.equal(y.view(torch.int64), ref.view(torch.int64)))
            allres[name]["warm_us"].append(warm)
            allres[name]["cold_us"].append(cold)
            allres[name]["b2b_us"].append(b2b)
            line[name] = {"warm_us": round(warm, 2), "cold_us": round(cold, 2), "b2b_us": round(b2b, 2),
                          "warm_gbs": round(nb / warm / 1e3, 1)}
        print(json.dumps(line), flush=True)
    summ = {"n": args.n, "nnz": A.nnz, "spmv_bytes": nbytes, "readwrite_bytes": rw_bytes, "bit_exact": exact}
    for name, r in allres.items():
        nb = variants[name][1]
        w = min(r["warm_us"])
        summ[name] = {"warm_us_min": round(w, 2), "warm_us_mean": round(sum(r["warm_us"]) / len(r["warm_us"]), 2),
                      "cold_us_mean": round(sum(r["cold_us"]) / len(r["cold_us"]), 2),
                      "b2b_us_mean": round(sum(r["b2b_us"]) / len(r["b2b_us"]), 2),
                      "warm_gbs_best": round(nb / w / 1e3, 1), "frac_of_8000_best": round(nb / w / 1e3 / 8000, 3)}
    print(json.dumps({"summary": summ}), flush=True)
    # the bench's own SpMV section (bench.spmv_bench) on the same matrix, in this process
    sys.path.insert(0, ROOT)
    from bench import spmv_bench
    del buf, flush, spacer
    torch.cuda.empty_cache()
    r = spmv_bench(A, gen)
    print(json.dumps({"bench_spmv_section": {k: r[k] for k in ("csr_us", "csr_us_graph", "csr_us_eager", "sell_us")},
                      "calibration": r.get("calibration")}), flush=True)


if __name__ == "__main__":
    main()
