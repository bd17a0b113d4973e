"""Per-apply kernel timeline from a rocprofv3 kernel trace: for the Chebyshev-4 apply (one apply = from one first-F-solve
fused-init sweep to the next), the span, the summed kernel time and each kernel's duration and the gap before it.

    python tools/apply_gaps.py gpurun_out/<tag>/prof/run_kernel_trace.csv
"""
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return n[5:] if n.startswith("void ") else n


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    first = [i for i, r in enumerate(rows) if "k_march_init" in r["Kernel_Name"] and "BNone" in r["Kernel_Name"]
             and "EpiChebFirstT<true, false, true, false>" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == 262144]
    spans = []
    for a, b in zip(first, first[1:]):
        s, e = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:b])
        spans.append((e - s, busy, a, b))
    spans.sort()
    print(f"{len(spans)} applies; fastest spans (us, kernel-busy us):",
          [(round(s / 1e3, 1), round(k / 1e3, 1)) for s, k, _, _ in spans[:6]])
    _, _, a, b = spans[len(spans) // 4]
    prev = None
    print("| kernel | us | gap before (us) |\n|---|---|---|")
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"| {short(r['Kernel_Name'])[:100]} | {(e - s) / 1e3:.1f} | {((s - prev) / 1e3) if prev else 0:.1f} |")
        prev = e


if __name__ == "__main__":
    main(sys.argv[1])
