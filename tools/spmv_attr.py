"""Attribute the CSR SpMV's HBM traffic (A u at 1024^2, k_csr_wave): the same matrix stream run with its x gathers
redirected into a 32 KB window (column j -> j mod 4096: the row structure, values and the kernel's path unchanged), so
FETCH_SIZE of that run is the matrix / row-structure / y part alone and the difference to the real run is what the
x gathers cost.  Run under rocprofv3 --pmc (tools/gpu.sh step spmvattr); the dispatches are REPS of the real A, then
REPS of the redirected copy, in that order.

    python tools/spmv_attr.py [--reps 10]                      (timing only)
    python tools/spmv_attr.py --reduce DIR                     (split DIR/pmc_{FETCH,WRITE}_SIZE CSVs, print JSON)
"""
import argparse
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KERNEL = "k_csr_wave<(anonymous namespace)::EpiStore>"


def run(reps):
    import torch
    import mp_block_preconditioners_amd as mp
    from mp_block_preconditioners_amd.csr import DeviceCSR
    bp = mp.MultiphaseBlockPreconditioner(1024, 1.0, 100.0, 1.0, device="cuda:0")
    A = bp.get_big_A_matrix(c=1.0, d_u=-1.0)[0]
    Aw = DeviceCSR(A.row_ptr, torch.remainder(A.col_idx, 4096).to(torch.int32), A.val, A.shape,
                   row_ptr_host=A.row_ptr_host)
    Aw.row_groups = A.row_groups   # the same block order (cell-range-major across the 5 fields)
    x = torch.randn(A.shape[1], dtype=torch.float64, device="cuda", generator=torch.Generator(device="cuda").manual_seed(0))
    y = torch.empty(A.shape[0], dtype=torch.float64, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    out = {"nnz": A.nnz, "rows": A.shape[0], "reps": reps}
    for name, M in (("A", A), ("A_x_window", Aw)):
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(reps):
            M.matvec(x, out=y)
        ev[1].record()
        torch.cuda.synchronize()
        out[name + "_us"] = ev[0].elapsed_time(ev[1]) * 1e3 / reps
    print(json.dumps(out), flush=True)


def reduce(d):
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = [r for r in csv.DictReader(open(os.path.join(d, f"pmc_{c}", "pmc_counter_collection.csv")))
                if r["Counter_Name"] == c and KERNEL in r["Kernel_Name"] and int(r["Grid_Size"]) > 4 * 1024 * 1024]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        half = len(rows) // 2
        for name, part in (("A", rows[:half]), ("A_x_window", rows[half:])):
            v = [float(r["Counter_Value"]) * 1024 for r in part]
            res.setdefault(name, {})[c.lower() + "_bytes"] = sum(v) / len(v) if v else None
    for name in res:
        f, w = res[name].get("fetch_size_bytes"), res[name].get("write_size_bytes")
        if f is not None and w is not None:
            res[name]["traffic_corrected"] = 2 * f + w   # MI355X_MICROARCH.md: FETCH_SIZE reads half of a wide stream
    if "A" in res and "A_x_window" in res:
        res["x_gather_traffic"] = res["A"]["traffic_corrected"] - res["A_x_window"]["traffic_corrected"]
        res["x_algorithmic_bytes"] = 5 * 1024 * 1024 * 8
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--reduce")
    a = ap.parse_args()
    reduce(a.reduce) if a.reduce else run(a.reps)
