"""seprate_point_cloud's batched FPS over zero-padded ragged clouds equals
the reference's per-sample FPS calls (utils/helpers.py:62-123) -- checked on
the oracle (the kernel is bit-exact to it, tests/test_gpu_pointops.py)."""
import numpy as np

from oracle import oracle as O


def test_zero_tail_padding_is_exact():
    rng = np.random.default_rng(3)
    B, N, M = 3, 3000, 512
    pts = (rng.random((B, N, 3)) - 0.5).astype(np.float32)
    pts[:, :, 2] += 0.2   # keep every real point outside the |p|^2 <= 1e-3 skip ball
    lens = [1200, 2999, 700]
    padded = np.zeros_like(pts)
    for b, n in enumerate(lens):
        padded[b, :n] = pts[b, :n]
    got = O.furthest_point_sample(padded, M)
    for b, n in enumerate(lens):
        ref = O.furthest_point_sample(np.ascontiguousarray(pts[b:b + 1, :n]), M)
        np.testing.assert_array_equal(got[b:b + 1], ref)
