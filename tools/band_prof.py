"""Where a rank's band hierarchy (distributed.LocalHierarchy) spends its setup time: one process builds rank `rank`'s
bands of the F or Gt_G hierarchy of an n^2 grid split over `world` ranks (no collectives are involved up to the
gathered level), timing every step with a device synchronisation.

    python tools/band_prof.py [--n 2048] [--world 4] [--rank 0] [--op F|GtG]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--op", default="F", choices=["F", "GtG"])
    a = ap.parse_args()
    import torch
    import mp_block_preconditioners_amd as mpb
    from mp_block_preconditioners_amd import _lib
    from mp_block_preconditioners_amd.csr import spgemm
    from mp_block_preconditioners_amd.distributed import (RowPartition, _relabel_cols, mg_bands, mg_part_cap)
    from mp_block_preconditioners_amd.mg import FIELDS_PRESSURE, FIELDS_VELOCITY, level_sizes, transfer_rows
    dev = torch.device("cuda")
    t = {}
    last = [time.perf_counter()]

    def stamp(name):
        torch.cuda.synchronize()
        now = time.perf_counter()
        t[name] = round(t.get(name, 0.0) + now - last[0], 4)
        last[0] = now
    fields = FIELDS_VELOCITY if a.op == "F" else FIELDS_PRESSURE
    part = RowPartition(a.n, a.world, a.rank, ghosts=True)
    bp = mpb.MultiphaseBlockPreconditioner(a.n, 1.0, 100.0, 1.0, device=dev)
    stamp("init")
    sizes = level_sizes(a.n, 16)
    cap = mg_part_cap(sizes, part, len(fields))
    S = mg_bands(sizes, fields, part, cap, dev)
    stamp("bands")
    if a.op == "F":
        A = bp.assemble_rows(_lib.OP_F, S[0], c=1.0, d_u=-1.0)
    else:
        Db = bp.assemble_rows(_lib.OP_D, S[0], c=1.0, d_u=-1.0)
        stamp("level0_D_rows")
        Gb = bp.assemble_rows(_lib.OP_G, torch.unique(Db.col_idx), global_shape=True, c=1.0, d_u=-1.0)
        stamp("level0_G_rows")
        A = spgemm(Db, Gb, alpha=-1.0)
    stamp("level0")
    info = {"sizes": sizes, "cap": cap, "band_rows": [int(s.numel()) for s in S]}
    for l in range(cap):
        C = torch.unique(A.col_idx)
        stamp(f"l{l}_unique")
        Pl = transfer_rows(sizes[l], fields, _lib.MG_P, C)
        stamp(f"l{l}_P_rows")
        Al = _relabel_cols(A, C)
        stamp(f"l{l}_relabel_A")
        AP = spgemm(Al, Pl)
        stamp(f"l{l}_AP")
        R = transfer_rows(sizes[l], fields, _lib.MG_R, S[l + 1])
        stamp(f"l{l}_R_rows")
        Rl = _relabel_cols(R, S[l])
        stamp(f"l{l}_relabel_R")
        A = spgemm(Rl, AP)
        stamp(f"l{l}_RAP")
        info[f"l{l}_nnz"] = [int(Al.nnz), int(AP.nnz), int(A.nnz)]
    print(json.dumps({"n": a.n, "world": a.world, "rank": a.rank, "op": a.op, **info, "seconds": t}), flush=True)


if __name__ == "__main__":
    main()
