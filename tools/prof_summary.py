"""Summarise a rocprofv3 --kernel-trace CSV per (kernel, grid size): calls, mean/min/max duration.

    python tools/prof_summary.py gpurun_out/<tag>/prof/run_kernel_trace.csv [--out profiles/x.md]
    python tools/prof_summary.py gpurun_out/<tag>/prof/run_results.db        (rocprofv3's default SQLite output)

The per-grid split separates launches of one template over different matrices (e.g. the
Chebyshev sweep over F, 4N rows, from the one over Gt_G, N rows), which rocprofv3 --stats lumps
together; bench.py's HIP-event average of the F sweep is checked against the F-grid row here.
"""
import argparse
import collections
import csv
import re


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0] if "(" in name else name[:120]   # the full template name, without the arguments


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out")
    args = ap.parse_args()
    agg = collections.defaultdict(list)
    if args.trace.endswith(".db"):
        import sqlite3
        db = sqlite3.connect(args.trace)
        for name, start, end, gx, wx in db.execute("select name, start, end, grid_x, workgroup_x from kernels"):
            agg[(short(name), int(gx), int(wx))].append(int(end) - int(start))
    else:
        for r in csv.DictReader(open(args.trace)):
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            agg[(short(r["Kernel_Name"]), int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))].append(d)
    total = sum(sum(v) for v in agg.values())
    lines = ["| kernel | grid (threads) | block | calls | mean us | min us | max us | % time |",
             "|---|---|---|---|---|---|---|---|"]
    for (k, g, b), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| {k} | {g} | {b} | {len(v)} | {sum(v) / len(v) / 1e3:.1f} | {min(v) / 1e3:.1f} | "
                     f"{max(v) / 1e3:.1f} | {100 * sum(v) / total:.1f} |")
    text = "\n".join(lines)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
