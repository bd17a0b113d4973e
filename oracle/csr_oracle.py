"""TEST INFRASTRUCTURE ONLY -- ctypes front-end of oracle/csr_oracle.c (sequential CPU checker).

See csr_oracle.c for the reference file:line each function restates.  The
shared object is built by ``oracle/Makefile`` (``__graft_entry__.build()`` runs it).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import scipy.sparse as sp

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libcsr_oracle.so")
_lib = None

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_D = ctypes.c_double


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "csr_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_spmv.argtypes = [_I32, _P, _P, _P, _P, _P]
        L.oracle_spmv_epi.argtypes = [_I32, _P, _P, _P, _P, _P, _P, _I32]
        L.oracle_jacobi_init.argtypes = [_I32, _P, _P, _P, _P]
        L.oracle_jacobi_step.argtypes = [_I32, _P, _P, _P, _P, _P, _P, _P, _P]
        L.oracle_cheb_init.argtypes = [_I32, _P, _P, _D, _P, _P, _P]
        L.oracle_cheb_step.argtypes = [_I32, _P, _P, _P, _P, _P, _P, _D, _D, _P, _P, _P]
        L.oracle_spgemm_count.argtypes = [_I32, _P, _P, _P, _P, _P, _P, _P]
        L.oracle_spgemm_count.restype = ctypes.c_int64
        L.oracle_spgemm_fill.argtypes = [_I32, _P, _P, _P, _P, _P, _P, _D, _P, _P, _P]
        L.oracle_spgemm_fill.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _csr(m):
    m = sp.csr_matrix(m)
    return (np.ascontiguousarray(m.indptr, dtype=np.int32),
            np.ascontiguousarray(m.indices, dtype=np.int32),
            np.ascontiguousarray(m.data, dtype=np.float64))


def _vec(x):
    return np.ascontiguousarray(x, dtype=np.float64)


def spmv(A, x, z=None, mode=0):
    """mode 0: A x ; 1: A x + z ; 2: z - A x  (sequential CSR-order sums)."""
    rp, ci, va = _csr(A)
    x = _vec(x)
    y = np.empty(A.shape[0], dtype=np.float64)
    zz = _vec(z) if z is not None else None
    lib().oracle_spmv_epi(A.shape[0], _p(rp), _p(ci), _p(va), _p(x), _p(zz), _p(y), mode)
    return y


def jacobi_init(b, diag, sub=None):
    b, diag = _vec(b), _vec(diag)
    out = np.empty_like(b)
    lib().oracle_jacobi_init(b.size, _p(b), _p(diag), _p(None if sub is None else _vec(sub)), _p(out))
    return out


def jacobi_step(A, xin, b, diag, sub=None):
    rp, ci, va = _csr(A)
    xin, b, diag = _vec(xin), _vec(b), _vec(diag)
    out = np.empty(A.shape[0], dtype=np.float64)
    lib().oracle_jacobi_step(A.shape[0], _p(rp), _p(ci), _p(va), _p(xin), _p(b), _p(diag),
                             _p(None if sub is None else _vec(sub)), _p(out))
    return out


def cheb_init(b, diag, c2, d, sub=None):
    b, diag = _vec(b), _vec(diag)
    out = np.empty_like(b)
    lib().oracle_cheb_init(b.size, _p(b), _p(diag), c2, _p(d), _p(None if sub is None else _vec(sub)),
                           _p(out))
    return out


def cheb_step(A, xin, b, diag, c1, c2, d, sub=None):
    rp, ci, va = _csr(A)
    xin, b, diag = _vec(xin), _vec(b), _vec(diag)
    out = np.empty(A.shape[0], dtype=np.float64)
    lib().oracle_cheb_step(A.shape[0], _p(rp), _p(ci), _p(va), _p(xin), _p(b), _p(diag), c1, c2,
                           _p(d), _p(None if sub is None else _vec(sub)), _p(out))
    return out


def spgemm(A, B, alpha=1.0):
    """alpha * (A @ B) keeping every structural product, columns sorted."""
    arp, aci, ava = _csr(A)
    brp, bci, bva = _csr(B)
    nrows = A.shape[0]
    row_nnz = np.empty(nrows, dtype=np.int32)
    tot = lib().oracle_spgemm_count(nrows, _p(arp), _p(aci), _p(ava), _p(brp), _p(bci), _p(bva),
                                    _p(row_nnz))
    if tot < 0:
        raise RuntimeError("spgemm row too wide for the oracle")
    crp = np.zeros(nrows + 1, dtype=np.int32)
    np.cumsum(row_nnz, out=crp[1:])
    cci = np.empty(int(tot), dtype=np.int32)
    cva = np.empty(int(tot), dtype=np.float64)
    rc = lib().oracle_spgemm_fill(nrows, _p(arp), _p(aci), _p(ava), _p(brp), _p(bci), _p(bva),
                                  float(alpha), _p(crp), _p(cci), _p(cva))
    if rc != 0:
        raise RuntimeError("spgemm fill failed")
    return sp.csr_matrix((cva, cci, crp), shape=(A.shape[0], B.shape[1]))
