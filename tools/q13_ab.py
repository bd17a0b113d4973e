"""Time the Gt_F_G diamond SpMV (mpbp_q13_spmv) at 1024^2 with HIP events (libmpbp from MPBP_LIB, for A/B builds).

    MPBP_LIB=mp-block-preconditioners_amd/lib/variants/libmpbp_<v>.so python tools/q13_ab.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(n=1024, reps=50):
    import torch
    import mp_block_preconditioners_amd as mp
    from mp_block_preconditioners_amd._lib import check, lib, ptr, stream_handle
    bp = mp.MultiphaseBlockPreconditioner(n, 1.0, 100.0, 1.0)
    _, _, F, D, G = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    _, GtFG = bp.commutator_products(F, D, G)
    vals = torch.empty(13 * n * n, dtype=torch.float64, device="cuda")
    check(lib().mpbp_q13_build(ctypes.byref(GtFG.cstruct()), n, ptr(vals), stream_handle()))
    x = torch.randn(n * n, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    ref = GtFG.matvec(x)
    check(lib().mpbp_q13_spmv(n, ptr(vals), 0, ptr(x), None, ptr(y), stream_handle()))
    assert torch.equal(y, ref)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(5):
        check(lib().mpbp_q13_spmv(n, ptr(vals), 0, ptr(x), None, ptr(y), stream_handle()))
    ev[0].record()
    for _ in range(reps):
        check(lib().mpbp_q13_spmv(n, ptr(vals), 0, ptr(x), None, ptr(y), stream_handle()))
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3 / reps
    nbytes = 13 * 8 * n * n + 2 * 8 * n * n
    print(json.dumps({"lib": os.environ.get("MPBP_LIB", "default"), "q13_us": us, "gbs": nbytes / us / 1e3}))


if __name__ == "__main__":
    main()
