"""CPU tests: the parity oracle against the reference's golden vectors and
against an independent literal simulation of the reference's FPS block."""
import numpy as np
import pytest

from conftest import golden
from oracle import oracle as O


def _tiled(rng, B, n_unique, N):
    u = (rng.random((B, n_unique, 3)) - 0.5).astype(np.float32)
    idx = np.r_[np.arange(n_unique), rng.integers(0, n_unique, N - n_unique)]
    return np.ascontiguousarray(u[:, idx, :])


def test_opt_n_threads_matches_cuda_utils():
    # cuda_utils.h:15-19
    for n, t in [(1, 1), (2, 2), (3, 2), (100, 64), (128, 128), (511, 256), (512, 512), (16384, 512)]:
        assert O.opt_n_threads(n) == t


@pytest.mark.parametrize(
    "B,N,M",
    [(2, 2048, 64), (2, 100, 30), (1, 513, 40), (1, 37, 20), (1, 8, 8), (2, 1024, 200)],
)
def test_fps_closed_form_equals_block_simulation(B, N, M):
    rng = np.random.default_rng(N * 7 + M)
    x = (rng.random((B, N, 3)) - 0.5).astype(np.float32)
    np.testing.assert_array_equal(O.furthest_point_sample(x, M), O.furthest_point_sample(x, M, blocksim=True))


def test_fps_ties_and_skipped_points_equal_block_simulation():
    rng = np.random.default_rng(3)
    x = _tiled(rng, 2, 300, 1024)  # more samples than unique points: exact ties at distance 0
    np.testing.assert_array_equal(O.furthest_point_sample(x, 600), O.furthest_point_sample(x, 600, blocksim=True))
    y = (rng.random((2, 1024, 3)) - 0.5).astype(np.float32)
    y[:, -64:] = 0.0  # |p|^2 <= 1e-3 points are never selected (sampling_gpu.cu:100-101)
    y[:, 5] = 0.01
    a = O.furthest_point_sample(y, 1000)
    np.testing.assert_array_equal(a, O.furthest_point_sample(y, 1000, blocksim=True))
    assert not np.isin(np.arange(960, 1024), a[:, 1:]).any()


def test_fps_properties():
    rng = np.random.default_rng(5)
    x = (rng.random((2, 700, 3)) - 0.5).astype(np.float32)
    idx = O.furthest_point_sample(x, 300)
    assert (idx[:, 0] == 0).all()
    for b in range(2):
        assert len(set(idx[b].tolist())) == 300  # unique while points remain
        # greedy property: each pick maximises the min distance to the picked set
        p = x[b].astype(np.float64)
        picked = [0]
        mind = ((p - p[0]) ** 2).sum(-1)
        for j in range(1, 50):
            assert np.isclose(mind[idx[b, j]], mind.max(), rtol=1e-5)
            mind = np.minimum(mind, ((p - p[idx[b, j]]) ** 2).sum(-1))


def test_chamfer_oracle_matches_reference_python():
    g = golden("chamfer.npz")
    for name in ["c1", "unit", "tiled"]:
        d1, d2, i1, i2 = O.chamfer_forward(g[name + "_a"], g[name + "_b"])
        # metrics/CD/unit_test.py:22-33 criteria
        assert ((d1 - g[name + "_d1"]) ** 2).mean() + ((d2 - g[name + "_d2"]) ** 2).mean() < 1e-8
        np.testing.assert_allclose(d1, g[name + "_d1"], atol=1e-7, rtol=0)
        np.testing.assert_array_equal(i1, g[name + "_i1"])
        np.testing.assert_array_equal(i2, g[name + "_i2"])


def _nm_distance_literal(a, b):
    """NmDistanceKernel (chamfer3D.cu:12-134) as a literal loop: 512-target chunks, the chunk
    seeded by its first target (`k==0 || d<best`), merged by `k2==0 || result>best`."""
    n, m = len(a), len(b)
    res, ri = [0.0] * n, [0] * n
    for j in range(n):
        x1, y1, z1 = (float(v) for v in a[j])
        for k2 in range(0, m, 512):
            best, best_i = 0.0, 0
            for k in range(min(m, k2 + 512) - k2):
                x2, y2, z2 = float(b[k2 + k][0]) - x1, float(b[k2 + k][1]) - y1, float(b[k2 + k][2]) - z1
                d = x2 * x2 + y2 * y2 + z2 * z2
                if k == 0 or d < best:
                    best, best_i = d, k + k2
            if k2 == 0 or res[j] > best:
                res[j], ri[j] = best, best_i
    return np.array(res, np.float32), np.array(ri, np.int32)


def test_chamfer_oracle_nonfinite_scan_order():
    """NaN at a chunk start: chunk 0's NaN seed pins (NaN, 0), a later chunk's hides that chunk;
    NaN elsewhere, inf points and non-finite queries.  Small-integer coordinates, so every
    distance is exact and the literal float64 loop is the reference's fp32 arithmetic."""
    rng = np.random.default_rng(17)
    B, N, M = 4, 70, 1100
    a = rng.integers(0, 8, (B, N, 3)).astype(np.float32)
    b = rng.integers(0, 8, (B, M, 3)).astype(np.float32)
    b[0, 0, 1] = np.nan                   # dir 0, chunk 0 seed
    b[1, 512, 0] = np.nan                 # dir 0, chunk 1 seed: chunk 1 hidden
    b[1, 1024, 2] = np.inf
    a[1, 0, 2] = np.nan                   # dir 1, chunk 0 seed
    b[2, 513] = np.nan                    # not a seed: skipped alone
    b[2, 0, 0] = np.inf
    a[2, 3] = [np.inf, 0.0, 0.0]          # inf query
    a[3, 5, 1] = np.nan                   # NaN query
    b[3, 1024, 1] = np.nan                # dir 0, chunk 2 seed (the short last chunk)
    d1, d2, i1, i2 = O.chamfer_forward(a, b)
    for bi in range(B):
        rd1, ri1 = _nm_distance_literal(a[bi], b[bi])
        rd2, ri2 = _nm_distance_literal(b[bi], a[bi])
        np.testing.assert_array_equal(d1[bi], rd1)
        np.testing.assert_array_equal(i1[bi], ri1)
        np.testing.assert_array_equal(d2[bi], rd2)
        np.testing.assert_array_equal(i2[bi], ri2)
    assert np.isnan(d1[0]).all() and (i1[0] == 0).all()
    assert np.isnan(d2[1]).all()


def test_chamfer_backward_oracle_matches_finite_differences():
    rng = np.random.default_rng(9)
    a = (rng.random((1, 40, 3))).astype(np.float32)
    b = (rng.random((1, 30, 3))).astype(np.float32)
    d1, d2, i1, i2 = O.chamfer_forward(a, b)
    w1 = rng.random(d1.shape).astype(np.float32)
    w2 = rng.random(d2.shape).astype(np.float32)
    g1, g2 = O.chamfer_backward(a, b, w1, w2, i1, i2)
    a64, b64 = a.astype(np.float64), b.astype(np.float64)
    # analytic gradient of sum(w1*d1)+sum(w2*d2) with the argmins held fixed
    e1 = np.zeros_like(a64)
    e2 = np.zeros_like(b64)
    for j in range(40):
        v = 2 * w1[0, j] * (a64[0, j] - b64[0, i1[0, j]])
        e1[0, j] += v
        e2[0, i1[0, j]] -= v
    for j in range(30):
        v = 2 * w2[0, j] * (b64[0, j] - a64[0, i2[0, j]])
        e2[0, j] += v
        e1[0, i2[0, j]] -= v
    np.testing.assert_allclose(g1, e1, atol=1e-5)
    np.testing.assert_allclose(g2, e2, atol=1e-5)


def test_knn_oracle_matches_reference_bitexact():
    k = golden("knn.npz")
    np.testing.assert_array_equal(O.knn(k["qk_new"], k["qk_xyz"], 16), k["qk_idx"])
    np.testing.assert_array_equal(O.knn(k["qk_new"], k["qk_xyz"], 16, pad=1), k["qk_idx_noself"])
    for name, K in [("kp3", 16), ("kp64", 8), ("kp256", 4)]:
        x = k[name + "_x"]
        np.testing.assert_array_equal(O.knn(x, x, K), k[name + "_idx"])
    np.testing.assert_array_equal(O.knn(k["kp3_x"], k["kp3_x"], 16), k["gl_idx"])


def test_knn_oracle_distance_formula_bitexact_and_ties():
    k = golden("knn.npz")
    sq = O.square_distance(k["qkt_new"][:, :16], k["qkt_xyz"])
    np.testing.assert_array_equal(sq, k["qkt_sqd"])
    # tiled input: argsort (unstable) orders exact ties arbitrarily; the
    # distance at every rank must still agree bit-for-bit.
    idx, d = O.knn(k["qkt_new"], k["qkt_xyz"], 16, return_dist=True)
    full = O.square_distance(k["qkt_new"], k["qkt_xyz"])
    dref = np.take_along_axis(full, k["qkt_idx"].astype(np.int64), -1)
    np.testing.assert_array_equal(dref, d)
    # and the oracle's own tie order is (distance, index) ascending
    for b in range(idx.shape[0]):
        for s in range(0, idx.shape[1], 37):
            pairs = list(zip(d[b, s].tolist(), idx[b, s].tolist()))
            assert pairs == sorted(pairs)


def test_depth_oracle_matches_reference_bitexact():
    g = golden("depth.npz")
    img = O.points2depth(g["points"], g["rot"], g["trans"])
    np.testing.assert_array_equal(img, g["img"])


def test_grid_oracle_matches_reference():
    g = golden("grid.npz")
    grid = O.points2grid(g["points_t"])
    np.testing.assert_array_equal(grid, g["grid"])
    img = O.grid2image(g["grid"], g["kern"])
    np.testing.assert_allclose(img[:, 0], g["img0"], atol=1e-6)
    np.testing.assert_array_equal(img[:, 0], img[:, 1])


def test_emd_oracle_properties():
    rng = np.random.default_rng(11)
    x1 = rng.random((2, 256, 3)).astype(np.float32)
    x2 = rng.random((2, 256, 3)).astype(np.float32)
    dist, ass = O.emd(x1, x2, 0.005, 200)
    assert (ass >= 0).all() and (ass < 256).all()
    # dist is the squared distance to the assigned point (CalcDist)
    ref = ((x1 - np.take_along_axis(x2, ass[..., None].astype(np.int64), 1)) ** 2).sum(-1)
    np.testing.assert_allclose(dist, ref, rtol=1e-5, atol=1e-7)
    # the auction converges to a (near) bijection: far better than random matching
    assert np.sqrt(dist).mean() < 0.6 * np.sqrt(((x1[:, :, None] - x2[:, None]) ** 2).sum(-1)).mean()
    assert min(len(np.unique(ass[b])) for b in range(2)) > 200
    # identical clouds: identity assignment
    d0, a0 = O.emd(x1, x1.copy(), 0.005, 50)
    assert (a0 == np.arange(256)).mean() > 0.95 and d0.max() < 1e-2


def test_ball_query_and_three_nn_oracle_semantics():
    rng = np.random.default_rng(12)
    xyz = rng.random((1, 64, 3)).astype(np.float32)
    new = xyz[:, :8].copy()
    idx = O.ball_query(0.3, 5, xyz, new)
    for j in range(8):
        d = ((xyz[0] - new[0, j]) ** 2).sum(-1)
        hits = np.nonzero(d < np.float32(0.3) ** 2)[0][:5]
        exp = np.full(5, hits[0])
        exp[: len(hits)] = hits
        np.testing.assert_array_equal(idx[0, j], exp)
    far = np.full((1, 1, 3), 10, np.float32)
    assert (O.ball_query(0.1, 4, xyz, far) == 0).all()  # no hit -> zeros
    dist, i3, d2 = O.three_nn(new, xyz)
    full = ((new[0, :, None] - xyz[0, None]) ** 2).sum(-1)
    np.testing.assert_array_equal(i3[0], np.argsort(full, -1, kind="stable")[:, :3])


def test_fps_prefix_property_oracle():
    """FPS is greedy: the first m indices of an M-point FPS are the m-point FPS of the same cloud
    (the basis of the models' shared partial-cloud FPS, model_utils.SharedFPS)."""
    rng = np.random.default_rng(7)
    x = (rng.random((3, 2048, 3)) - 0.5).astype(np.float32)
    x[1, 1024:] = x[1, :1024]   # exact duplicates: ties decided by the tie rule alone
    full = O.furthest_point_sample(x, 1024)
    np.testing.assert_array_equal(full[:, :512], O.furthest_point_sample(x, 512))
