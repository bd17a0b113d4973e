"""Summarise the bench.py lines of an A/B run (tools/gpu.sh ab:...): applies/s and the F-sweep average per variant.

    python tools/ab_table.py gpurun_out/<tag>
"""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "ab_bench_*.log"))):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            r = d["roofline"]
            print(f"{os.path.basename(f)[9:-4]:32s} {d['value']:8.1f} applies/s   F sweep {r['avg_launch_us']:6.1f} us")
