"""CPU checks of the C-ABI library: it loads, exports every symbol include/mpbp.h declares, and its
host-only entry points (row-block planner, Chebyshev coefficients, operator sizes) agree with the
oracle.  No compute kernels are launched (there is no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def _header_symbols():
    with open(os.path.join(ROOT, "include", "mpbp.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(mpbp_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from mp_block_preconditioners_amd import _lib
    L = _lib.lib()
    declared = _header_symbols()
    assert len(declared) >= 25
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    assert set(declared) == set(_lib.exported_symbols())
    assert L.mpbp_version().decode().startswith("libmpbp")


def test_library_is_gfx950_code_object():
    from mp_block_preconditioners_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_operator_sizes():
    from mp_block_preconditioners_amd import _lib
    L = _lib.lib()
    n = 7
    N = n * n
    expect = {_lib.OP_A: (5 * N, 5 * N), _lib.OP_F: (4 * N, 4 * N), _lib.OP_D: (N, 4 * N),
              _lib.OP_G: (4 * N, N), _lib.OP_L_N: (2 * N, 2 * N), _lib.OP_D_S: (N, 2 * N),
              _lib.OP_G_N: (2 * N, N), _lib.OP_XI_S: (2 * N, 2 * N)}
    for op, (r, c) in expect.items():
        assert L.mpbp_stokes_rows(n, op) == r
        assert L.mpbp_stokes_cols(n, op) == c
    assert L.mpbp_stokes_rows(n, 99) < 0
    assert b"unknown operator" in L.mpbp_last_error()


def _py_plan(rp, a, b, max_rows=256, cap=4095):
    out = []
    r = a
    while r < b:
        s = e = r
        while e < b and e - s < max_rows and rp[e + 1] - rp[s] <= cap:
            e += 1
        if e == s:
            e = s + 1
        out.append((s, e))
        r = e
    return out


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_row_block_planner(seed):
    from mp_block_preconditioners_amd import _lib
    rng = np.random.default_rng(seed)
    lengths = rng.integers(0, 40, size=3000)
    lengths[rng.integers(0, 3000, size=3)] = 5000          # rows longer than the LDS stage
    rp = np.zeros(lengths.size + 1, dtype=np.int32)
    np.cumsum(lengths, out=rp[1:])
    L = _lib.lib()
    for a, b in ((0, 3000), (17, 2900), (5, 5)):
        need = L.mpbp_plan_row_blocks(rp.ctypes.data_as(ctypes.c_void_p), a, b, None, 0)
        buf = np.zeros(2 * max(need, 1), dtype=np.int32)
        L.mpbp_plan_row_blocks(rp.ctypes.data_as(ctypes.c_void_p), a, b, buf.ctypes.data_as(ctypes.c_void_p), need)
        got = [tuple(p) for p in buf[: 2 * need].reshape(-1, 2)]
        assert got == _py_plan(rp, a, b)
        for s, e in got:
            assert e - s <= 256 and (rp[e] - rp[s] <= 4095 or e - s == 1)


def test_cheb_coeffs_match_oracle():
    from mp_block_preconditioners_amd import _lib
    from oracle.schur_oracle import cheb_coeffs
    L = _lib.lib()
    for lmin, lmax, k in ((0.05, 2.0, 8), (1e-3, 1.7, 3), (0.0, 1.0, 1)):
        c1 = np.zeros(k)
        c2 = np.zeros(k)
        assert L.mpbp_cheb_coeffs(lmin, lmax, k, c1.ctypes.data_as(ctypes.c_void_p),
                                  c2.ctypes.data_as(ctypes.c_void_p)) == 0
        o1, o2 = cheb_coeffs(lmin, lmax, k)
        assert np.array_equal(c1, o1) and np.array_equal(c2, o2)
    c = np.zeros(2)
    assert L.mpbp_cheb_coeffs(1.0, 1.0, 2, c.ctypes.data_as(ctypes.c_void_p), c.ctypes.data_as(ctypes.c_void_p)) < 0


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from mp_block_preconditioners_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "libmpbp.so"))
    with pytest.raises(_lib.MpbpError, match="no CPU fallback"):
        _lib.lib()


def test_wave_table_flags():
    """The row blocks' wave table (csr.wave_table, mpbp_rowblocks.table) on the host: wave entry ranges from row_ptr, and
    the uniform flag exactly for the 64-row waves of 8 / 10 / 12 entries each from an even offset."""
    import numpy as np
    from mp_block_preconditioners_amd.csr import wave_table
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 20, size=1000)
    lens[0:64] = 12          # uniform wave, even start
    lens[64:128] = 10
    lens[128:192] = 7        # uniform but not 8 / 10 / 12
    lens[256:320] = 8
    lens[300] = 9            # broken
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    pairs = np.array([[0, 256], [256, 512], [512, 700], [700, 1000]], dtype=np.int32)
    t = wave_table(rp, pairs).reshape(-1, 8)
    assert np.array_equal(t[:, 0], pairs[:, 0]) and np.array_equal(t[:, 1], pairs[:, 1])
    for b, (ra, rb) in enumerate(pairs):
        for w in range(5):
            assert t[b, 2 + w] == rp[min(ra + 64 * w, rb)]
        for w in range(4):
            a = ra + 64 * w
            L = lens[a:a + 64]
            want = int(L[0]) if (rb - a >= 64 and np.all(L == L[0]) and L[0] in (8, 10, 12) and rp[a] % 2 == 0) else 0
            assert (int(t[b, 7]) >> (8 * w)) & 255 == want, (b, w)
    assert (int(t[0, 7]) & 255) == 12 and ((int(t[0, 7]) >> 8) & 255) == (10 if rp[64] % 2 == 0 else 0)


def test_kernel_options_block_lifetime_and_reentry():
    """kernel_options (host-only, mpbp_kernel_opts_set_thread): the installed struct stays referenced while the block is
    active -- the C thread-local pointer refers to it -- and a second entry of the same instance is refused, so the
    previous choice can always be restored."""
    from mp_block_preconditioners_amd import _lib
    base = _lib.kernel_opts()
    ko = _lib.kernel_options(march_rows=7)
    with ko as o:
        assert any(x is o for x in _lib._INSTALLED)
        assert _lib.kernel_opts().march_rows == 7
        with pytest.raises(RuntimeError):
            ko.__enter__()
        with _lib.kernel_options(march_rows=3):
            assert _lib.kernel_opts().march_rows == 3
        assert _lib.kernel_opts().march_rows == 7
    assert not any(x is o for x in _lib._INSTALLED)
    assert _lib.kernel_opts().march_rows == base.march_rows
