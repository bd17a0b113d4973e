"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (over bench.py's apply, tools/gpu.sh (step pmc)) to HBM
bytes per F sweep launch -- the same launches bench.py's HIP events time.

    python tools/pmc_reduce.py gpurun_out/<tag> [--write profiles/pmc_traffic.json]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE
reads exactly half of a wide (16 B/lane) coalesced stream, so the read side is doubled here
("corrected"); WRITE_SIZE is exact for 16 B/lane streaming stores (ours are 8 B/lane -- uncalibrated,
reported as read).  Both raw and corrected numbers are kept.
"""
import argparse
import csv
import json
import os


def mean_counter(path, counter, kernel_substr, grid, first=None):
    rows = []
    for r in csv.DictReader(open(path)):
        parts = kernel_substr if isinstance(kernel_substr, tuple) else (kernel_substr,)
        if r["Counter_Name"] == counter and all(k in r["Kernel_Name"] for k in parts) and \
                (grid is None or int(r["Grid_Size"]) == grid):
            rows.append((int(r.get("Dispatch_Id", 0) or 0), float(r["Counter_Value"])))
    rows.sort()
    vals = [v for _, v in (rows[:first] if first else rows)]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--write")
    args = ap.parse_args()
    grid = 4 * args.n * args.n
    # F sweep kernels and their launch grids (threads)
    # (the marching kernel's grid depends on its rows per workgroup: matched by name only)
    # (the F policy may carry the parameter identities: FStencilDev or FStencilDevM<M>)
    # "stencil": the first F solve's plain sweeps (b streamed, no sub: EpiChebT<true, false, SD, false>), the
    # launches bench.py's `roofline` times; tools/gpu.sh's pmc step writes them under pmc_apply_<counter>
    kernels = {"stencil": (("k_march<(anonymous namespace)::FStencilDev", "(anonymous namespace)::XPlain, ",
                            "EpiChebT<true, false, ", "BNone>"), args.n * args.n // 4),   # 4 rows x 256 cols / WG
               "sell": ("k_sell_rows<(anonymous namespace)::EpiCheb>", grid),   # grid 4N: F rows, not Gt_G
               # round 4: the whole-solve F launch (the first solve: b streamed, no sub; the second: G x_p, sub), the
               # fused Gt_G solve and Gt_F_G on the diamond -- every kernel of the default apply but D
               # (round 6: k_fsolve_w, the 32 x 16 tile form -- kernel option f_solve_tile 1, the default)
               "fsolve": (("k_fsolve_w<32, 16, 3, false, false, (anonymous namespace)::BNone>",), None),
               "fsolve_gx": (("k_fsolve_w<32, 16, 3, true, false, (anonymous namespace)::GxBT<false> >",), None),
               "gtg_solve_drhs": (("k_gtg_solve<3, false, 512, true>",), None),      # the first: rhs = D Y + v_p inside
               "gtg_solve": (("k_gtg_solve<3, false, 512, false>",), None),
               "q13": (("k_q13<(anonymous namespace)::EpiStore, ",), None)}
    out = {"n": args.n, "source": args.run_dir}
    for lay, (kname, kgrid) in kernels.items():
        res = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            f = os.path.join(args.run_dir, f"pmc_{lay}_{c}", "pmc_counter_collection.csv")
            if lay not in ("sell",) and not os.path.exists(f):
                f = os.path.join(args.run_dir, f"pmc_apply_{c}", "pmc_counter_collection.csv")
            if os.path.exists(f):
                res[c] = mean_counter(f, c, kname, kgrid)
        if "FETCH_SIZE" in res and res["FETCH_SIZE"][0] is not None and "WRITE_SIZE" in res:
            fetch = res["FETCH_SIZE"][0] * 1024
            write = res["WRITE_SIZE"][0] * 1024
            out[lay] = {"fetch_bytes_raw": fetch, "write_bytes": write, "dispatches": res["FETCH_SIZE"][1],
                        "traffic_bytes_corrected": 2 * fetch + write, "traffic_bytes_raw": fetch + write}
    # the plain A SpMV (apply.py:72) of tools/spmv_ab.py, both layouts' product kernels
    spmv_k = {"csr_spmv_A": "k_csr_wave<(anonymous namespace)::EpiStore>",
              "sell_spmv_A": "k_sell_rows<(anonymous namespace)::EpiStore>"}
    # tools/spmv_ab.py runs the default k_csr_wave first (5 warmup + REPS launches), then the variants that share its
    # kernel name (no wave table, plain row-order blocks: the latter re-fetches x across XCDs): only the default's
    # launches count (round 4: averaging all of them had reported 1.07x the algorithmic bytes)
    first = {"csr_spmv_A": 15, "sell_spmv_A": None}
    for key, kname in spmv_k.items():
        res = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            f = os.path.join(args.run_dir, f"pmc_spmv_{c}", "pmc_counter_collection.csv")
            if os.path.exists(f):
                res[c] = mean_counter(f, c, kname, None, first[key])
        if res.get("FETCH_SIZE", (None,))[0] is not None and res.get("WRITE_SIZE", (None,))[0] is not None:
            fetch = res["FETCH_SIZE"][0] * 1024
            write = res["WRITE_SIZE"][0] * 1024
            out[key] = {"fetch_bytes_raw": fetch, "write_bytes": write, "dispatches": res["FETCH_SIZE"][1],
                        "traffic_bytes_corrected": 2 * fetch + write, "traffic_bytes_raw": fetch + write}
    # calibration on a known byte count in the same runs: k_cheb_init over F's 4N rows reads b, diag and
    # writes d, x with 8-B lanes -- exactly 2 x 8 x 4N bytes each way (f_mode=assembled pass only)
    cal = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = os.path.join(args.run_dir, f"pmc_sell_{c}", "pmc_counter_collection.csv")
        if os.path.exists(f):
            cal[c] = mean_counter(f, c, "k_cheb_init", grid)
    if cal.get("FETCH_SIZE", (None,))[0] is not None and cal.get("WRITE_SIZE", (None,))[0] is not None:
        want = 2 * 8 * grid
        out["calibration_k_cheb_init"] = {
            "expected_read_bytes": want, "expected_write_bytes": want,
            "fetch_bytes_raw": cal["FETCH_SIZE"][0] * 1024, "fetch_x2_over_expected": 2 * cal["FETCH_SIZE"][0] * 1024 / want,
            "write_bytes": cal["WRITE_SIZE"][0] * 1024, "write_over_expected": cal["WRITE_SIZE"][0] * 1024 / want}
    print(json.dumps(out, indent=1))
    if args.write:
        with open(args.write, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
