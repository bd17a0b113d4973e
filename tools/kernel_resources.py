"""Per-kernel VGPRs / scratch / occupancy of libmpbp for gfx950 (compiler resource-usage remarks).

    python tools/kernel_resources.py [name-substring ...]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.environ.get("MPBP_SRC") or os.path.join(ROOT, "mp-block-preconditioners_amd", "csrc", "mpbp.hip")


def main():
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "-fno-fast-math", "-I" + os.path.join(ROOT, "include"), "--offload-device-only", "-c", SRC,
           "-o", "/tmp/_mpbp_res.o", *os.environ.get("MPBP_FLAGS", "").split(), "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark: +(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).split()[0]] = int(m.group(2))
    demangled = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows),
                               capture_output=True, text=True).stdout.splitlines()
    keys = sys.argv[1:]
    for r, d in zip(rows, demangled):
        d = d.replace("(anonymous namespace)::", "")
        if keys and not any(k in d for k in keys):
            continue
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('SGPRs', '?'):>4} sgpr {r.get('ScratchSize', '?'):>4} scratch occ {r.get('Occupancy', '?')}  {d[:150]}")


if __name__ == "__main__":
    main()
