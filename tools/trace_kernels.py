"""Per-kernel-instance durations from a rocprofv3 --kernel-trace CSV (full template names, so every k_march
instance is its own row), sorted by total time.

    python tools/trace_kernels.py gpurun_out/<tag>/prof/run_kernel_trace.csv [--match k_march] [--md out.md]
"""
import argparse
import collections
import csv
import re


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return re.sub(r"\((?!anonymous).*", "", name)[:120]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", default="")
    ap.add_argument("--md")
    args = ap.parse_args()
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(args.csv)):
        k = short(r["Kernel_Name"])
        if args.match in k:
            d[(k, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines = ["| kernel | grid | calls | mean us | min us | max us | total us |", "|---|---|---|---|---|---|---|"]
    for (k, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| {k} | {g} | {len(v)} | {sum(v) / len(v):.1f} | {min(v):.1f} | {max(v):.1f} | {sum(v):.0f} |")
    print("\n".join(lines))
    if args.md:
        open(args.md, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
