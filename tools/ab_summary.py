"""One line per bench JSON in gpurun_out/TAG/ab_bench_*.log: apply rate and time, both k_fsolve launches, the
multigrid apply and its roofline kernel.

    python tools/ab_summary.py TAG
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag):
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", tag, "ab_bench_*.log"))):
        name = os.path.basename(f)[len("ab_bench_"):-4]
        for line in open(f):
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            r, r2 = d["roofline"], d.get("roofline_second_f_solve") or {}
            m = d.get("mg_apply") or {}
            mr = m.get("roofline") or {}
            print(f"{name:28s} {d['value']:8.1f}/s {d['ms_per_step'] * 1e3:7.1f} us  fs1 {r['avg_launch_us']:6.1f}"
                  f"  fs2 {r2.get('avg_launch_us', 0):6.1f}  mg {m.get('ms_per_step', 0):6.3f} ms"
                  f"  mgk {mr.get('avg_launch_us', 0):6.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
