"""Per-kernel mean of every counter in rocprofv3 --pmc passes (one directory per pass under a run directory).

    python tools/pmc_table.py gpurun_out/<tag> [--match k_march] [--json out.json]

Kernels are keyed by their full name (template arguments kept, so each F-sweep instance is its own row); values
are per-dispatch means.  Derived columns when the counters are present: VALU instructions per wave, the fraction
of wave cycles spent waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES), and VALU-busy cycles per SIMD.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name)[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--match", default="")
    ap.add_argument("--json")
    args = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(args.run_dir, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if args.match in k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in sorted(acc.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        m["dispatches"] = max(len(v) for v in cs.values())
        if "SQ_INSTS_VALU" in m and m.get("SQ_WAVES"):
            m["valu_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
        if "SQ_WAIT_ANY" in m and m.get("SQ_WAVE_CYCLES"):
            m["wait_frac"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
        out[k] = m
        print(k)
        print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(m.items())))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
