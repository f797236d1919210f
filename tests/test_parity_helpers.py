"""The parity helpers themselves (CPU): the scaled contract and SURVEY §8(d)'s
per-element measure, and which entries count as cancellation entries."""
import numpy as np

import parity
from phdslam.types import GAUSSIAN2D


def _map(rows):
    m = np.zeros(len(rows), GAUSSIAN2D)
    for i, (w, mx, my, c) in enumerate(rows):
        m[i]["weight"] = w
        m[i]["mean"] = (mx, my)
        m[i]["cov"] = c
    return m


def test_elementwise_counts_cancellation_entries_apart():
    A = _map([(0.5, 10.0, 0.2, (4.0, 1e-3, 1e-3, 9.0)), (0.25, -3.0, 7.0, (1.0, 0.0, 0.0, 1.0))])
    B = A.copy()
    # an off-diagonal produced by cancellation moves by 1e-3 of itself, 1e-7 of the matrix
    B[0]["cov"][1] = np.float32(1e-3 * (1 + 1e-3))
    B[0]["cov"][2] = B[0]["cov"][1]
    # a mean near the origin moves by 1e-4 of itself (1e-7 of the position)
    B[0]["mean"][1] = np.float32(0.2 * (1 + 1e-4))
    strict = [0.0, 0, 0, 0, 0.0]
    ok, worst = parity.compare_maps(A, B, 1e-5, strict)
    assert ok and worst < 1e-5
    assert strict[1] == 3 and strict[2] == 14  # three entries beyond the per-element measure ...
    assert strict[3] == 0  # ... all of them cancellation entries


def test_elementwise_flags_diagonals_weights_and_far_means():
    A = _map([(0.5, 10.0, 0.2, (4.0, 1e-3, 1e-3, 900.0))])
    for field, idx, val in (("cov", 0, 4.0 * (1 + 5e-5)), ("weight", None, 0.5 * (1 + 5e-5)),
                            ("mean", 0, 10.0 * (1 + 5e-5))):
        B = A.copy()
        if idx is None:
            B[0][field] = np.float32(val)
        else:
            B[0][field][idx] = np.float32(val)
        strict = [0.0, 0, 0, 0, 0.0]
        parity.compare_maps(A, B, 1e-5, strict)
        assert strict[3] == 1, field
        assert strict[4] > 1e-5


def test_noncancellation_mask():
    fa = np.array([[0.1, 0.5, 3.0, 1.0, 0.2, 0.2, 2.0]])
    m = parity.noncancellation_mask(fa, fa)
    assert m.tolist() == [[True, False, True, True, False, False, True]]
