"""One line per bench JSON log: applies/s, F-sweep us, roofline frac, SpMV GB/s.  python tools/bench_table.py LOG..."""
import json
import sys

for f in sys.argv[1:]:
    try:
        line = [x for x in open(f) if x.startswith("{")][-1]
    except (OSError, IndexError):
        print(f"{f}: no JSON line")
        continue
    d = json.loads(line)
    r = d["roofline"]
    cs = d.get("roofline_csr_spmv") or {}
    print(f"{f:60s} {d['value']:8.1f} applies/s  sweep {r['avg_launch_us']:6.2f} us  frac {r['frac']:.3f}  "
          f"csr {cs.get('achieved', 0):7.1f} GB/s (frac {cs.get('frac', 0):.3f}, sell frac {cs.get('sell_frac') or 0:.3f})")
