"""Comparison helpers for GPU-vs-oracle parity (tolerances per SURVEY.md §8(d))."""
import numpy as np
from scipy.optimize import linear_sum_assignment

RTOL = 1e-5


def close(a, b, rtol=RTOL, floor=1e-30, scale=None):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    ref = np.maximum(np.abs(a), np.abs(b))
    if scale is not None:
        ref = np.maximum(ref, scale)
    return np.abs(a - b) <= rtol * ref + floor


def _fields(X):
    return np.concatenate([X["weight"][:, None], X["mean"], X["cov"]], 1).astype(np.float64)


def match_maps(A, B):
    """Match two GM maps (GAUSSIAN2D arrays) as multisets. Returns (ia, ib) index arrays.
    Fast path: both sorted by (mean x, mean y, weight) pair up element by element
    when every pair agrees to 1e-4 of its scale; otherwise (near-equal keys in a
    different order) an optimal assignment."""
    if len(A) != len(B):
        raise AssertionError(f"map sizes differ: {len(A)} vs {len(B)}")
    if len(A) == 0:
        return np.zeros(0, int), np.zeros(0, int)
    ia = np.lexsort((A["weight"], A["mean"][:, 1], A["mean"][:, 0]))
    ib = np.lexsort((B["weight"], B["mean"][:, 1], B["mean"][:, 0]))
    fa, fb = _fields(A[ia]), _fields(B[ib])
    scale = np.maximum(np.maximum(np.abs(fa), np.abs(fb)), 1e-3)
    if np.all(np.abs(fa - fb) <= 1e-4 * scale):
        return ia, ib
    ma = np.stack([A["mean"][:, 0], A["mean"][:, 1]], 1).astype(np.float64)
    mb = np.stack([B["mean"][:, 0], B["mean"][:, 1]], 1).astype(np.float64)
    cost = np.sum((ma[:, None, :] - mb[None, :, :]) ** 2, -1)
    cost += (np.log(np.maximum(A["weight"], 1e-30))[:, None].astype(np.float64)
             - np.log(np.maximum(B["weight"], 1e-30))[None, :].astype(np.float64)) ** 2
    ia, ib = linear_sum_assignment(cost)
    return ia, ib


def compare_maps(A, B, rtol=RTOL, strict=None):
    """Return (ok, worst_rel) for two maps compared as multisets.  strict: a list
    [worst, count, elements, count_noncancel, worst_noncancel] that accumulates
    SURVEY.md §8(d)'s per-element measure of the same matching (elementwise)."""
    ia, ib = match_maps(A, B)
    a, b = A[ia], B[ib]
    if strict is not None:
        sw, sn, st, snc, swn = _elementwise(a, b, full=True)
        strict[0] = max(strict[0], sw)
        strict[1] += sn
        strict[2] += st
        strict[3] += snc
        strict[4] = max(strict[4], swn)
    # covariance entries relative to the matrix scale (off-diagonals can be ~0)
    sa = np.sqrt(np.abs(a["cov"][:, 0] * a["cov"][:, 3]))[:, None]
    ok_w = close(a["weight"], b["weight"], rtol, floor=1e-12)
    mscale = np.maximum(np.abs(a["mean"]).max(1, keepdims=True), 1.0)
    ok_m = close(a["mean"], b["mean"], rtol, scale=mscale)
    ok_c = close(a["cov"], b["cov"], rtol, scale=sa)
    worst = max(_rel(a["weight"], b["weight"]), _rel(a["mean"], b["mean"], mscale), _rel(a["cov"], b["cov"], sa))
    return bool(ok_w.all() and ok_m.all() and ok_c.all()), worst


def elementwise(A, B):
    """SURVEY.md §8(d)'s per-element measure beside compare_maps' scaled one:
    (worst |a-b| / max(|a|,|b|) over every field of every matched component,
    number of elements with |a-b| > RTOL max(|a|,|b|) + 1e-30, elements compared).
    The contract is compare_maps' (DESIGN.md §2): an entry produced by
    cancellation (a covariance off-diagonal or a mean near 0) moves by more than
    1e-5 of itself when an input moves by an ulp, while the matrix or the
    position it belongs to moves by 1e-7 of its scale."""
    ia, ib = match_maps(A, B)
    return _elementwise(A[ia], B[ib])


# fields of _fields(): weight, mean x, mean y, cov 00, 01, 10, 11.  An entry is
# a "cancellation entry" when it is a covariance off-diagonal (a sum of terms of
# both signs) or a mean coordinate with |x| < 1 (near the origin); every other
# entry — weights, covariance diagonals, means away from the origin — is held
# to SURVEY §8(d)'s per-element measure itself (noncancellation_mask).
_OFFDIAG = np.array([False, False, False, False, True, True, False])
_MEAN = np.array([False, True, True, False, False, False, False])


def noncancellation_mask(fa, fb):
    big = np.maximum(np.abs(fa), np.abs(fb)) >= 1.0
    return ~_OFFDIAG[None, :] & (~_MEAN[None, :] | big)


def _elementwise(a, b, full=False):
    fa, fb = _fields(a), _fields(b)
    ref = np.maximum(np.abs(fa), np.abs(fb))
    d = np.abs(fa - fb)
    rel = np.where(ref > 0, d / np.maximum(ref, 1e-300), 0.0)
    beyond = d > RTOL * ref + 1e-30
    out = (float(rel.max()) if rel.size else 0.0, int(np.sum(beyond)), int(rel.size))
    if not full:
        return out
    nc = noncancellation_mask(fa, fb)
    worst_nc = float(rel[nc].max()) if nc.any() else 0.0
    return out + (int(np.sum(beyond & nc)), worst_nc)


def unmatched(A, B, rtol=RTOL):
    """Components of A and of B left without a partner that agrees within the
    tolerances of compare_maps (one-to-one, greedy in A order).  Used for
    particles with near-threshold prune / merge decisions: every component those
    decisions do not touch must still match.  Returns (n_unmatched_A, n_unmatched_B)."""
    if len(A) == 0 or len(B) == 0:
        return len(A), len(B)
    wb = B["weight"].astype(np.float64)
    mb = B["mean"].astype(np.float64)
    cb = B["cov"].astype(np.float64)
    used = np.zeros(len(B), bool)
    miss = 0
    for i in range(len(A)):
        wa = np.float64(A["weight"][i])
        ma = A["mean"][i].astype(np.float64)
        ca = A["cov"][i].astype(np.float64)
        sa = np.sqrt(abs(ca[0] * ca[3]))
        ms = max(np.abs(ma).max(), 1.0)
        ok = (~used & (np.abs(wb - wa) <= rtol * np.maximum(np.abs(wb), abs(wa)) + 1e-12)
              & np.all(np.abs(mb - ma) <= rtol * np.maximum(np.maximum(np.abs(mb), np.abs(ma)), ms), 1)
              & np.all(np.abs(cb - ca) <= rtol * np.maximum(np.maximum(np.abs(cb), np.abs(ca)), sa) + 1e-30, 1))
        j = np.flatnonzero(ok)
        if len(j):
            used[j[0]] = True
        else:
            miss += 1
    return miss, int((~used).sum())


def _rel(a, b, scale=None):
    if len(a) == 0:
        return 0.0
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    ref = np.maximum(np.abs(a), np.abs(b))
    if scale is not None:
        ref = np.maximum(ref, scale)
    ref = np.maximum(ref, 1e-30)
    return float(np.max(np.abs(a - b) / ref))
