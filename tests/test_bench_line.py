"""bench.py's printed line (CPU): the contract's keys, north_star's CSR SpMV target last, and the whole line inside the
8 KB of stdout the driver records -- checked on the full record of a round-5 run (profiles/r05zc_bench.json)."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _full_record():
    lines = [ln for ln in open(os.path.join(ROOT, "profiles", "r05zc_bench.json")) if ln.startswith("{")]
    return json.loads(lines[-1])


def test_compact_line_fits_the_driver_tail_with_the_csr_target_last():
    full = _full_record()
    line = bench.compact_line(full)
    text = json.dumps(line)
    assert len(text) < 6000, len(text)
    for k in CONTRACT:
        assert k in line, k
    assert list(line)[-1] == "roofline_csr_spmv"
    cs = line["roofline_csr_spmv"]
    assert cs["frac"] == bench._r(full["roofline_csr_spmv"]["frac"])
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(cs)
    # the tail the driver keeps (8 183 characters in round 5) holds the whole object
    assert '"roofline_csr_spmv"' in text[-8000:]
    # every solve_level run survives, as one row
    assert len(line["solve_level"]["runs"]) == len(full["solve_level"]["runs"])
    assert line["roofline"]["avg_launch_us"] == bench._r(full["roofline"]["avg_launch_us"])


def test_compact_line_without_optional_sections():
    full = _full_record()
    for k in ("spmv_A", "roofline_csr_spmv", "mg_apply", "solve_level", "time_to_solution", "host_buffer_matvec"):
        full[k] = None
    full["cpu_baseline"] = None
    line = bench.compact_line(full)
    assert line["cpu_baseline"] is None and line["vs_baseline"] is None   # contract keys stay, even when null
    assert "roofline_csr_spmv" not in line and "mg_apply" not in line
