"""TEST INFRASTRUCTURE ONLY -- CPU restatement of libmpbp's FGMRES vector kernels.

The reference's outer solve is pyamg.krylov.fgmres (solve.py:285; pyamg 5.x, absent here): classical Gram-Schmidt
Arnoldi with Givens rotations over dot products and axpys.  mp-block-preconditioners_amd/solve.py runs it with

* ``mpbp_rdot`` -- reproducible inner products by binned summation (Demmel & Nguyen, "Fast reproducible floating-point
  summation", ARITH 2013: pre-rounding every term against a common extractor sigma = 1.5 * 2^e so that the partial
  sums of each fold are exact), 3 folds, extractor exponents from a bound on the terms;
* ``mpbp_gs_update`` -- w - V^T h with the basis vectors added in order;

* ``mpbp_gs_update_rdot`` -- CGS2's first update and second projection fused, the extractors from an a-priori bound;
* ``mpbp_rdot2`` / ``mpbp_dcgs2_update`` -- DCGS2's block product and its scalars and two updates (delayed
  re-orthogonalisation: Swirydowicz, Langou, Ananthan, Yang, Thomas, "Low synchronization Gram-Schmidt and GMRES
  algorithms", NLAA 2020; Bielich et al., "Low-synch Gram-Schmidt with delayed reorthogonalization for Krylov solvers",
  Parallel Computing 2022);

restated here in numpy: ``rd_sigmas`` / ``rdot_folds`` / ``rdot`` / ``gs_update`` / ``gs_update_rdot`` / ``rdot2_folds`` /
``dcgs2_coeffs`` / ``dcgs2_update``.  Because every fold sum is exact,
numpy's (pairwise) sum gives the same bits as the GPU's tree of partial sums, whatever the split of the vector.
``TorchKrylov`` has the KrylovKernels interface over CPU torch tensors (and a gloo group), so tests can drive the
product's fgmres host logic -- the distributed reductions, bounds, Givens rotations -- on the CPU.

Parity pinning: pyamg is absent, so nothing pins the iteration counts to the reference's solver ("parity unpinned");
these kernels are pinned to the GPU kernels bit for bit (tests/test_gpu_krylov.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch

FOLDS = 3


def rd_sigmas(bound: float, ntot: int) -> list[float]:
    """The 3 extractors for terms |t| <= bound over ntot terms (mpbp.hip rd_sigmas)."""
    if not math.isfinite(bound):
        return [float("nan")] * FOLDS
    if not bound > 0.0:
        return [0.0] * FOLDS
    m, E = math.frexp(bound)   # bound = m 2^E, 0.5 <= m < 1
    L = max(int(ntot), 1).bit_length() + 1
    if E + L > 1023:
        return [float("nan")] * FOLDS
    out = []
    for f in range(FOLDS):
        ex = E + (f + 1) * L - 53 * f
        out.append(math.ldexp(1.5, ex) if ex >= -1022 else 0.0)
    return out


def fold_terms(t: np.ndarray, sig) -> np.ndarray:
    """(FOLDS, len(t)): the pre-rounded parts q_f of every term (mpbp.hip rd_fold)."""
    r = np.asarray(t, dtype=np.float64).copy()
    q = np.zeros((FOLDS, r.size))
    for f, s in enumerate(sig):
        if s != 0.0:
            qf = (s + r) - s
            q[f] = qf
            r = r - qf
    return q


def rdot_folds(V: np.ndarray, w: np.ndarray, ntot: int, bv, bw: float) -> np.ndarray:
    """acc[3i + f]: the exact fold sums of V[i] . w."""
    V = np.atleast_2d(np.asarray(V, dtype=np.float64))
    acc = np.zeros(3 * V.shape[0])
    for i in range(V.shape[0]):
        sig = rd_sigmas(float(bv[i]) * float(bw), ntot)
        q = fold_terms(V[i] * w, sig)
        acc[3 * i: 3 * i + 3] = q.sum(axis=1)   # exact: the summation order does not matter
    return acc


def finish(acc) -> np.ndarray:
    a = np.asarray(acc, dtype=np.float64).reshape(-1, 3)
    return (a[:, 0] + a[:, 1]) + a[:, 2]


def rdot(V, w, ntot=None, bv=None, bw=None) -> np.ndarray:
    V = np.atleast_2d(np.asarray(V, dtype=np.float64))
    w = np.asarray(w, dtype=np.float64)
    ntot = w.size if ntot is None else ntot
    bv = np.max(np.abs(V), axis=1) if bv is None else bv
    bw = float(np.max(np.abs(w))) if bw is None else bw
    return finish(rdot_folds(V, w, ntot, bv, bw))


def gs_update(V, k, h, w) -> np.ndarray:
    """w - sum_i V[i] h[i], the products added in order i = 0 .. k-1 from 0.0 (mpbp.hip k_gs_update)."""
    a = np.zeros_like(np.asarray(w, dtype=np.float64))
    for i in range(k):
        a = a + V[i] * h[i]
    return w - a


def update_bound(bw: float, bv, h, k: int) -> float:
    """The a-priori bound on |w - V^T h| the fused CGS2 pass takes its extractors from (mpbp.hip k_gs_update_rdot):
    (max|w| + sum_i bv[i] |h[i]|, added in order) (1 + 2^-40)."""
    b = float(bw)
    for i in range(k):
        b = b + float(bv[i]) * abs(float(h[i]))
    return b * (1.0 + 2.0 ** -40)


def gs_update_rdot(V, k, h, w, ntot, bv, bw):
    """(w - V^T h, the fold sums of V[i] . (w - V^T h) under update_bound's extractors) (mpbp_gs_update_rdot)."""
    r = gs_update(V, k, h, w)
    return r, rdot_folds(np.atleast_2d(V)[:k], r, ntot, bv, update_bound(bw, bv, h, k))


def rdot2_folds(V, u, w, ntot, bv, bu: float, bw: float) -> np.ndarray:
    """mpbp_rdot2: the fold sums of V[i] . u (first 3k) and V[i] . w (next 3k)."""
    return np.concatenate([rdot_folds(V, u, ntot, bv, bu), rdot_folds(V, w, ntot, bv, bw)])


def dcgs2_coeffs(j: int, acc, bw: float):
    """mpbp.hip k_dcgs2_coeffs: (hu[0..j], hw[0..j], P = [r, 1/r, c, bound of u_{j+1}]) in the kernel's order."""
    k = j + 1
    a = np.asarray(acc, dtype=np.float64)
    hu = [(float(a[3 * i]) + float(a[3 * i + 1])) + float(a[3 * i + 2]) for i in range(k)]
    hw = [(float(a[3 * k + 3 * i]) + float(a[3 * k + 3 * i + 1])) + float(a[3 * k + 3 * i + 2]) for i in range(k)]
    ss, sz, b = 0.0, 0.0, float(bw)
    for i in range(j):
        ss = ss + hu[i] * hu[i]
        sz = sz + hu[i] * hw[i]
        b = b + abs(hw[i])
    r, rinv = 1.0, 1.0
    if j > 0:
        d = hu[j] - ss
        r = math.sqrt(d) if d > 0.0 else 0.0
        rinv = 1.0 / r if r > 0.0 else 0.0
    c = (hw[j] - sz) * rinv
    b = ((b + abs(c)) * rinv) * (1.0 + 2.0 ** -40)
    return np.asarray(hu), np.asarray(hw), np.asarray([r, rinv, c, b])


def dcgs2_update(V: np.ndarray, j: int, hu, hw, P, w, upd_w=True):
    """mpbp.hip k_dcgs2_update on a (>= j + 2) x n basis, in place: V[j] <- (V[j] - sum_i V[i] s_i) / r,
    V[j + 1] <- ((w - sum_i V[i] z_i) - V[j] c) / r, the sums over i < j in order from 0.0."""
    su = np.zeros(V.shape[1])
    sw = np.zeros(V.shape[1])
    for i in range(j):
        su = su + V[i] * hu[i]
        sw = sw + V[i] * hw[i]
    q = (V[j] - su) * P[1]
    V[j] = q
    if upd_w:
        V[j + 1] = ((np.asarray(w, dtype=np.float64) - sw) - q * P[2]) * P[1]


class TorchKrylov:
    """KrylovKernels' interface (solve.py) on CPU torch float64 tensors, optionally over a gloo group."""

    def __init__(self, n, kmax, device="cpu", group=None):
        self.n, self.kmax, self.group = int(n), int(kmax), group
        n_total = self.n
        if group is not None:
            import torch.distributed as dist
            self.dist = dist
            t = torch.tensor([self.n], dtype=torch.int64)
            dist.all_reduce(t, group=group)
            n_total = int(t.item())
        self.n_total = n_total
        self.acc = torch.zeros(3 * self.kmax, dtype=torch.float64)
        self.h = torch.zeros(self.kmax, dtype=torch.float64)

    def _reduce(self, t, op):
        if self.group is not None:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM if op == "sum" else self.dist.ReduceOp.MAX,
                                 group=self.group)
        return t

    def amax(self, x, out):
        out[0] = float(np.max(np.abs(x.numpy()))) if x.numel() else 0.0
        return self._reduce(out, "max")

    def fold_sums(self, V, ld, k, w, vb, wb):
        Vm = V.reshape(-1)[: k * ld].view(k, ld)[:, : self.n].numpy() if V.dim() == 1 else V[:k, : self.n].numpy()
        a = rdot_folds(Vm, w.numpy()[: self.n], self.n_total, vb.numpy()[:k], float(wb[0]))
        self.acc[: 3 * k] = torch.from_numpy(a)
        return self._reduce(self.acc[: 3 * k], "sum")

    def dots(self, V, ld, k, w, vb, wb):
        self.fold_sums(V, ld, k, w, vb, wb)
        self.h[:k] = torch.from_numpy(finish(self.acc[: 3 * k].numpy()))
        return self.h[:k]

    def update(self, V, ld, k, h, w, out):
        Vm = V.reshape(-1)[: k * ld].view(k, ld)[:, : self.n].numpy() if V.dim() == 1 else V[:k, : self.n].numpy()
        r = w.numpy().copy()
        for i0 in range(0, k, 256):   # solve.KrylovKernels: 256 basis rows per launch
            kc = min(256, k - i0)
            r = gs_update(Vm[i0:i0 + kc], kc, h.numpy()[i0:i0 + kc], r)
        out.copy_(torch.from_numpy(r))
        return out

    def block_folds(self, V, ld, k, u, w, vb, bu, bw):
        Vm = V[:k, : self.n].numpy()
        a = rdot2_folds(Vm, u.numpy()[: self.n], w.numpy()[: self.n], self.n_total, vb.numpy()[:k], float(bu[0]),
                        float(bw[0]))
        if not hasattr(self, "acc2"):
            self.acc2 = torch.zeros(6 * 256, dtype=torch.float64)
        self.acc2[: 6 * k] = torch.from_numpy(a)
        return self._reduce(self.acc2[: 6 * k], "sum")

    def dcgs2_update(self, V, ld, j, acc, bw, w, upd_w=True):
        hu, hw, P = dcgs2_coeffs(j, acc.numpy(), float(bw[0]))
        Vm = V.numpy()   # a view: updated in place
        dcgs2_update(Vm, j, hu, hw, P, w.numpy() if upd_w else None, upd_w)
        return torch.from_numpy(hu), torch.from_numpy(hw), torch.from_numpy(P)

    def update_dots(self, V, ld, k, h, w, vb, wb):
        """w <- w - V[:k]^T h in place, then h2 = V[:k] w under the a-priori bound (KrylovKernels.update_dots)."""
        Vm = V.reshape(-1)[: k * ld].view(k, ld)[:, : self.n].numpy() if V.dim() == 1 else V[:k, : self.n].numpy()
        r, a = gs_update_rdot(Vm, k, h.numpy()[:k], w.numpy()[: self.n], self.n_total, vb.numpy()[:k], float(wb[0]))
        w.copy_(torch.from_numpy(r))
        self.acc[: 3 * k] = torch.from_numpy(a)
        self._reduce(self.acc[: 3 * k], "sum")
        self.h[:k] = torch.from_numpy(finish(self.acc[: 3 * k].numpy()))
        return self.h[:k]
