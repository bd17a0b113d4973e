"""Static instruction mix of kernels in an assembly file (hipcc -save-temps output), by demangled-name substrings.

    python tools/isa_mix.py FILE.s "k_march<" "FStencilFast" "EpiChebT<true, false, true, false, true>"
"""
import collections
import re
import subprocess
import sys


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S+:", l)]
    for k, i in enumerate(starts):
        name = lines[i].split(":")[0]
        dn = subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
        if not all(p in dn for p in pats):
            continue
        end = starts[k + 1] if k + 1 < len(starts) else len(lines)
        c = collections.Counter()
        for l in lines[i + 1:end]:
            t = l.strip()
            if not l.startswith("\t") or not t or t.startswith((".", ";")):
                continue
            op = t.split()[0]
            if op.startswith("v_") and ("f64" in op or "fma" in op):
                c["v_f64"] += 1
            elif op.startswith("v_"):
                c["v_other"] += 1
            elif op.startswith("ds_read"):
                c["ds_read"] += 1
            elif op.startswith("ds_write"):
                c["ds_write"] += 1
            elif op.startswith(("global_load", "buffer_load")):
                c["vmem_load"] += 1
            elif op.startswith(("global_store", "buffer_store")):
                c["vmem_store"] += 1
            elif op.startswith("scratch_"):
                c["scratch"] += 1
            elif op.startswith("s_waitcnt"):
                c["waitcnt"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
            else:
                c["other"] += 1
        print(dn[:150])
        print("   ", dict(c), "total", sum(c.values()))


if __name__ == "__main__":
    main()
