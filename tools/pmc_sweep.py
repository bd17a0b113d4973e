"""Drive only the dominant kernel for rocprofv3 --pmc passes: K Chebyshev sweeps over F (1024^2).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o pmc -- python tools/pmc_sweep.py [--layout sell]

tools/pmc_reduce.py then divides the counters of the F-sweep dispatches by their count.
"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=1024)
    ap.add_argument("--sweeps", type=int, default=10)
    ap.add_argument("--layout", default="sell", choices=["sell", "csr", "stencil"])
    args = ap.parse_args()
    import torch
    import mp_block_preconditioners_amd as mp
    from mp_block_preconditioners_amd._lib import check, lib, ptr, stream_handle
    bp = mp.MultiphaseBlockPreconditioner(args.grid, 1.0, 100.0, 1.0)
    _, _, F, _, _ = bp.get_big_A_matrix(c=1.0, d_u=-1.0)
    diag = F.diagonal()
    S = F.to_sell()
    n = F.shape[0]
    g = torch.Generator(device="cuda").manual_seed(0)
    x, b, d = (torch.randn(n, dtype=torch.float64, device="cuda", generator=g) for _ in range(3))
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    for _ in range(args.sweeps):
        if args.layout == "stencil":
            st = F.stencil
            check(lib().mpbp_f_stencil_cheb_step(ctypes.byref(st.prm), ptr(st.cell), ptr(st.uface), ptr(st.vface),
                                                 None, ptr(x), ptr(b), 0.3, 1.1, ptr(d), None, ptr(y), stream_handle()))
        elif args.layout == "sell":
            check(lib().mpbp_sell_cheb_step(ctypes.byref(S.cstruct()), ptr(x), ptr(b), ptr(diag), 0.3, 1.1, ptr(d),
                                            None, ptr(y), stream_handle()))
        else:
            check(lib().mpbp_cheb_step(ctypes.byref(F.cstruct()), ctypes.byref(F.blocks.cstruct()), ptr(x), ptr(b),
                                       ptr(diag), 0.3, 1.1, ptr(d), None, ptr(y), stream_handle()))
        x, y = y, x
    torch.cuda.synchronize()
    print("nnz", F.nnz, "rows", n, "slices", S.nslices)


if __name__ == "__main__":
    main()
