"""Build experiment variants of libmpbp (compile-time switches) next to the product library.

    python tools/build_variants.py name=-DFLAG=1,-DOTHER=2 [name2=...]
    MPBP_LIB=mp-block-preconditioners_amd/lib/variants/libmpbp_<name>.so python bench.py ...

The product path (tests, smoke, bench defaults) always loads lib/libmpbp.so; variants are for A/B runs.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def build(spec):
    name, _, flags = spec.partition("=")
    out_dir = os.path.join(ge.PKG, "lib", "variants")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f"libmpbp_{name}.so")
    cmd = [ge.HIPCC, *ge.HIP_FLAGS, *[f for f in flags.split(",") if f], "-I", os.path.join(ROOT, "include"),
           *ge.SOURCES, "-o", out, *ge.LIBS]
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    with ThreadPoolExecutor(4) as ex:
        for o in ex.map(build, sys.argv[1:]):
            print(o)
