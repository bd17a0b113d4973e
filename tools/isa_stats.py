"""Instruction mix of one kernel in the gfx950 assembly of libmpbp.

    python tools/isa_stats.py <mangled-name-substring> [--top 40]
"""
import argparse
import collections
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--src", default=os.environ.get("MPBP_SRC") or
                    os.path.join(ROOT, "mp-block-preconditioners_amd", "csrc", "mpbp.hip"))
    args = ap.parse_args()
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                           "-fno-fast-math", "-I" + os.path.join(ROOT, "include"), "--offload-device-only", "-S",
                           args.src, "-o", "/tmp/_mpbp_isa.s"], stderr=subprocess.DEVNULL)
    L = open("/tmp/_mpbp_isa.s").read().split("\n")
    start = next(i for i, l in enumerate(L) if l.startswith(args.kernel) or (args.kernel in l and l.split(":")[0].endswith(
        args.kernel.split(":")[0]) and l.rstrip().split(";")[0].strip().endswith(":")))
    body = []
    for l in L[start + 1:]:
        if l.startswith(".Lfunc_end") or l.startswith("\t.section"):
            break
        t = l.strip()
        if l.startswith("\t") and t and not t.startswith((".", ";")):
            body.append(t.split()[0])
    c = collections.Counter(body)
    groups = collections.Counter()
    for k, v in c.items():
        g = ("v_*_f64" if k.startswith("v_") and "f64" in k else "valu-other" if k.startswith("v_") else
             "ds" if k.startswith("ds_") else "global" if k.startswith(("global_", "buffer_")) else
             "salu" if k.startswith("s_") else "other")
        groups[g] += v
    print("static instructions:", len(body), dict(groups))
    for k, v in c.most_common(args.top):
        print(f"{v:5d} {k}")


if __name__ == "__main__":
    main()
