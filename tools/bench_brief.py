"""One-screen summary of bench.py JSON lines (a log file with one line per run).

    python tools/bench_brief.py gpurun_out/<tag>/bench.log [...]
"""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if not line.startswith("{"):
            continue
        b = json.loads(line)
        r, r2, cs, mg = b["roofline"], b.get("roofline_second_f_solve") or {}, b.get("roofline_csr_spmv"), b.get("mg_apply")
        print(f"{f}: {b['value']:.0f} applies/s ({b['ms_per_step'] * 1e3:.1f} us) numerics={b['config'].get('f_numerics', '?')[:5]}"
              f" n_gpus={b['n_gpus']}")
        print(f"  dominant {r['kernel'][:60]}: {r['avg_launch_us']:.1f} us, {r['bytes_per_launch'] / 1e6:.1f} MB, "
              f"frac {r['frac']:.3f}; 2nd solve {r2.get('avg_launch_us', float('nan')):.1f} us")
        if cs:
            print(f"  csr A u: {cs['avg_launch_us']:.1f} us frac {cs['frac']:.3f} (b2b {cs['frac_back_to_back']:.3f})")
        if mg and "ms_per_step" in mg:
            print(f"  mg apply {mg['ms_per_step']:.3f} ms; {mg['roofline']['kernel'][:40]} {mg['roofline']['avg_launch_us']:.1f} us "
                  f"frac {mg['roofline']['frac']:.3f}")
        cpu = b.get("cpu_baseline")
        if cpu:
            print(f"  cpu {cpu['value']:.2f} applies/s parity {cpu.get('parity')} rel {cpu.get('rel_inf_vs_gpu')}")
        for k in ("eager_applies_per_s", "mg_apply_partitioned", "solve_distributed"):
            if k in b:
                print(f"  {k}: {b[k]}")
        sl = b.get("solve_level")
        if sl:
            for row in sl["runs"]:
                x = dict(zip(sl["cols"], row)) if isinstance(row, list) else row
                print(f"    solve n={x['n']} eta={x['eta_n']:g} {x['preconditioner']}: {x['iterations']} it "
                      f"{x['seconds']:.3f} s apply {x['apply_ms']} ms conv={x['converged']}")
