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


def match_maps(A, B):
    """Match two GM maps (GAUSSIAN2D arrays) as multisets. Returns (ia, ib) index arrays."""
    if len(A) != len(B):
        raise AssertionError(f"map sizes differ: {len(A)} vs {len(B)}")
    if len(A) == 0:
        return np.zeros(0, int), np.zeros(0, int)
    ma = np.stack([A["mean"][:, 0], A["mean"][:, 1]], 1).astype(np.float64)
    mb = np.stack([B["mean"][:, 0], B["mean"][:, 1]], 1).astype(np.float64)
    cost = np.sum((ma[:, None, :] - mb[None, :, :]) ** 2, -1)
    cost += (np.log(np.maximum(A["weight"], 1e-30))[:, None].astype(np.float64)
             - np.log(np.maximum(B["weight"], 1e-30))[None, :].astype(np.float64)) ** 2
    ia, ib = linear_sum_assignment(cost)
    return ia, ib


def compare_maps(A, B, rtol=RTOL):
    """Return (ok, worst_rel) for two maps compared as multisets."""
    ia, ib = match_maps(A, B)
    a, b = A[ia], B[ib]
    # covariance entries relative to the matrix scale (off-diagonals can be ~0)
    sa = np.sqrt(np.abs(a["cov"][:, 0] * a["cov"][:, 3]))[:, None]
    ok_w = close(a["weight"], b["weight"], rtol, floor=1e-12)
    mscale = np.maximum(np.abs(a["mean"]).max(1, keepdims=True), 1.0)
    ok_m = close(a["mean"], b["mean"], rtol, scale=mscale)
    ok_c = close(a["cov"], b["cov"], rtol, scale=sa)
    worst = max(_rel(a["weight"], b["weight"]), _rel(a["mean"], b["mean"], mscale), _rel(a["cov"], b["cov"], sa))
    return bool(ok_w.all() and ok_m.all() and ok_c.all()), worst


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
