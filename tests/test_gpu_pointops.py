"""GPU parity: libpcops.so (through the reference-shaped Python API) against
the CPU oracle and the reference's golden vectors.  Integer/index outputs are
compared bit-exactly; float outputs with the tolerance stated per test."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def T(a, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t if dtype is None else t.to(dtype)


def _tiled(rng, B, n_unique, N):
    u = (rng.random((B, n_unique, 3)) - 0.5).astype(np.float32)
    idx = np.r_[np.arange(n_unique), rng.integers(0, n_unique, N - n_unique)]
    return np.ascontiguousarray(u[:, idx, :])


# ------------------------------------------------------------------ FPS
FPS_CASES = [
    ("c1", 4, 2048, 512),
    ("gt", 2, 16384, 2048),
    ("n512", 3, 512, 128),
    ("merge", 2, 2304, 512),
    ("odd", 2, 513, 100),
    ("small", 3, 100, 40),
    ("tiny", 2, 37, 20),
    ("wave", 1, 64, 64),
    ("stream", 2, 20000, 300),
    # sizes between the step's shapes (register kernel instances and their edges)
    ("p4096", 2, 4096, 1024),
    ("p4097", 1, 4097, 900),
    ("p55", 2, 8192, 2048),
    ("p8193", 1, 8193, 1500),
    ("p3001", 1, 3001, 777),
]


@pytest.mark.parametrize("name,B,N,M", FPS_CASES)
def test_fps_bitexact(dev, name, B, N, M):
    from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample

    rng = np.random.default_rng(B * 1000 + N + M)
    x = (rng.random((B, N, 3)) - 0.5).astype(np.float32)
    got = furthest_point_sample(T(x, dev), M).cpu().numpy()
    np.testing.assert_array_equal(got, O.furthest_point_sample(x, M))


def test_fps_ties_and_zero_points_bitexact(dev):
    from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample

    rng = np.random.default_rng(1)
    x = _tiled(rng, 2, 700, 2048)  # PCN-style duplicates, M > unique -> exact ties
    got = furthest_point_sample(T(x, dev), 1024).cpu().numpy()
    np.testing.assert_array_equal(got, O.furthest_point_sample(x, 1024))
    y = (rng.random((2, 2048, 3)) - 0.5).astype(np.float32)
    y[:, -64:] = 0.0
    got = furthest_point_sample(T(y, dev), 2000).cpu().numpy()
    np.testing.assert_array_equal(got, O.furthest_point_sample(y, 2000))
    z = np.zeros((1, 1024, 3), np.float32)  # nothing valid -> index 0 everywhere
    assert (furthest_point_sample(T(z, dev), 16).cpu().numpy() == 0).all()


@pytest.mark.parametrize("kind", ["tiled16384", "zeros8192", "clusters", "line", "all_zero", "gauss16384"])
def test_fps_edge_cases_bitexact(dev, kind):
    """FPS on inputs that stress the tie order and the skip rule: more samples than
    distinct points (all running distances 0 -> the tie order alone decides),
    skipped |p|^2 <= 1e-3 points, far-apart clusters, a degenerate (flat) cloud,
    nothing valid at all."""
    from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample

    rng = np.random.default_rng(len(kind))
    if kind == "tiled16384":
        x, M = _tiled(rng, 2, 1500, 16384), 2048
    elif kind == "zeros8192":
        x, M = (rng.random((2, 8192, 3)) - 0.5).astype(np.float32), 8000
        x[:, -1000:] = 0.0
        x[:, 100:140] = 1e-2   # |p|^2 = 3e-4 <= 1e-3: skipped too
    elif kind == "clusters":
        x = (rng.standard_normal((2, 6000, 3)) * 1e-3).astype(np.float32)
        x[:, ::2] += 100.0
        x[:, 1::3] -= 50.0
        M = 1500
    elif kind == "line":
        x = np.zeros((1, 5000, 3), np.float32)
        x[0, :, 0] = np.linspace(-1, 1, 5000, dtype=np.float32)
        M = 600
    elif kind == "all_zero":
        x, M = np.zeros((1, 4096, 3), np.float32), 64
    else:
        x, M = (rng.standard_normal((4, 16384, 3)) * 0.45).astype(np.float32), 2048
    got = furthest_point_sample(T(x, dev), M).cpu().numpy()
    np.testing.assert_array_equal(got, O.furthest_point_sample(x, M))


@pytest.mark.parametrize("kind", ["tiled512", "tiled256", "zeros512", "all_zero512", "n513", "tiled64"])
def test_fps_wave_kernel_edge_cases_bitexact(dev, kind):
    """The one-wave kernel (clouds of <= 512 points, fps_wave_kernel) on the inputs
    that stress its re-implemented tie order and skip rule: padded
    partials with duplicated points and more samples than distinct points,
    skipped near-origin points, an all-zero cloud, and N = 513 (the first size
    past it)."""
    from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample

    rng = np.random.default_rng(100 + len(kind))
    if kind == "tiled512":
        x, M = _tiled(rng, 3, 90, 512), 128
    elif kind == "tiled256":
        x, M = _tiled(rng, 2, 40, 256), 200
    elif kind == "tiled64":
        x, M = _tiled(rng, 2, 9, 64), 64
    elif kind == "zeros512":
        x, M = (rng.random((2, 512, 3)) - 0.5).astype(np.float32), 400
        x[:, -100:] = 0.0
        x[:, 10:30] = 1e-2   # |p|^2 = 3e-4 <= 1e-3: skipped
    elif kind == "all_zero512":
        x, M = np.zeros((2, 512, 3), np.float32), 32
    else:
        x, M = _tiled(rng, 2, 200, 513), 300
    got = furthest_point_sample(T(x, dev), M).cpu().numpy()
    np.testing.assert_array_equal(got, O.furthest_point_sample(x, M))


@pytest.mark.parametrize("kind", ["tiled2304", "zeros4000", "all_zero2500", "n2049", "tiled4096", "gauss3001"])
def test_fps_mw_kernel_edge_cases_bitexact(dev, kind):
    """The 4-wave kernel (512-thread clouds of 5-8 points per reference thread, fps_mw_kernel:
    2048 < N <= 4096) on the inputs that stress its tie order across lanes, slots and waves:
    duplicated points with more samples than distinct points (the tie order alone decides),
    skipped near-origin points, an all-zero cloud, N = 2049 (the first size it takes) and 4096."""
    from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample

    rng = np.random.default_rng(200 + len(kind))
    if kind == "tiled2304":
        x, M = _tiled(rng, 3, 300, 2304), 1024
    elif kind == "tiled4096":
        x, M = _tiled(rng, 2, 500, 4096), 1024
    elif kind == "zeros4000":
        x, M = (rng.random((2, 4000, 3)) - 0.5).astype(np.float32), 3000
        x[:, -700:] = 0.0
        x[:, 50:90] = 1e-2   # |p|^2 = 3e-4 <= 1e-3: skipped
    elif kind == "all_zero2500":
        x, M = np.zeros((2, 2500, 3), np.float32), 40
    elif kind == "n2049":
        x, M = (rng.random((2, 2049, 3)) - 0.5).astype(np.float32), 700
    else:
        x, M = (rng.standard_normal((3, 3001, 3)) * 0.45).astype(np.float32), 777
    got = furthest_point_sample(T(x, dev), M).cpu().numpy()
    np.testing.assert_array_equal(got, O.furthest_point_sample(x, M))


def test_fps_full_size_properties(dev):
    """B=32, 16384 -> 2048 (the loss FPS): size-independent properties."""
    from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample

    g = torch.Generator(device="cpu").manual_seed(2)
    x = (torch.randn(32, 16384, 3, generator=g) * 0.45).to(dev)
    idx = furthest_point_sample(x, 2048).long()
    assert (idx[:, 0] == 0).all()
    assert all(len(torch.unique(idx[b])) == 2048 for b in range(32))
    # every one of the 32 clouds bit-exactly against the oracle
    np.testing.assert_array_equal(idx.cpu().numpy(), O.furthest_point_sample(x.cpu().numpy(), 2048))


@pytest.mark.parametrize("B,N,M,tail", [(16, 6144, 2048, "zero"), (5, 6144, 2048, "garbage"),
                                        (3, 2304, 1024, "garbage"), (2, 16384, 2048, "garbage"),
                                        (2, 20000, 300, "garbage"), (3, 400, 100, "garbage"),
                                        (4, 6144, 512, "edge")])
def test_fps_counts_bitexact(dev, B, N, M, tail):
    """pcops_furthest_point_sampling_counts (the batched crop's zero-padded clouds with known valid
    counts): equal to the plain FPS -- and to the oracle -- on the buffer whose rows >= count are
    zero, whatever the rows past the count hold ("garbage": they must be ignored); counts across
    slot boundaries, counts 0 and N, and counts below the block size ("edge")."""
    from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample, furthest_point_sample_counts

    rng = np.random.default_rng(B * N + M)
    x = (rng.random((B, N, 3)) - 0.5).astype(np.float32)
    if tail == "edge":
        counts = np.array([0, N, 1, 300][:B], np.int32)
    else:
        counts = rng.integers(max(1, N // 3), N + 1, B).astype(np.int32)
        counts[0] = N
        if B > 2:
            counts[1] = (N // 512) * 512 if N >= 512 else N // 2   # an exact slot boundary
    z = x.copy()
    for b in range(B):
        z[b, counts[b]:] = 0.0
    if tail == "zero":
        x = z.copy()
    got = furthest_point_sample_counts(T(x, dev), T(counts, dev), M).cpu().numpy()
    ref = furthest_point_sample(T(z, dev), M).cpu().numpy()
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(got, O.furthest_point_sample(z, M))


@pytest.mark.parametrize("B,N,M,m", [(4, 2048, 1024, 512), (32, 2048, 512, 512), (3, 2048, 1024, 256),
                                     (2, 16384, 2048, 256)])
def test_fps_prefix_property(dev, B, N, M, m):
    """The models' shared partial-cloud FPS (model_utils.SharedFPS) rests on FPS being greedy: the
    first m indices of an M-point FPS are the m-point FPS of the same cloud.  Bitwise, on plain and
    on tiled (PCN-style duplicate, tie-heavy) clouds, and through SharedFPS.take on a side stream."""
    from svdformer_pointsea_amd import _lib
    from svdformer_pointsea_amd.model_utils import SharedFPS
    from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample

    rng = np.random.default_rng(B + N + M + m)
    for x in ((rng.random((B, N, 3)) - 0.5).astype(np.float32), _tiled(rng, B, N // 3, N)):
        xt = T(x, dev)
        full = furthest_point_sample(xt, M)
        np.testing.assert_array_equal(full[:, :m].cpu().numpy(), furthest_point_sample(xt, m).cpu().numpy())
        with _lib.fork(dev, inputs=(xt,)):
            sh = SharedFPS(furthest_point_sample(xt, M))
        got = sh.take(m)
        np.testing.assert_array_equal(got.cpu().numpy(), full[:, :m].cpu().numpy())


# ------------------------------------------------------------------ gather / group
def test_gather_and_grad(dev):
    from svdformer_pointsea_amd.pointnet2_utils import gather_operation

    rng = np.random.default_rng(3)
    f = rng.standard_normal((3, 64, 2048)).astype(np.float32)
    idx = rng.integers(0, 2048, (3, 512)).astype(np.int32)
    ft = T(f, dev).requires_grad_(True)
    out = gather_operation(ft, T(idx, dev))
    np.testing.assert_array_equal(out.detach().cpu().numpy(), O.gather_operation(f, idx))
    go = rng.standard_normal(out.shape).astype(np.float32)
    out.backward(T(go, dev))
    np.testing.assert_allclose(ft.grad.cpu().numpy(), O.gather_operation_grad(go, idx, 2048), rtol=1e-6, atol=1e-6)


def test_group_and_grad(dev):
    from svdformer_pointsea_amd.pointnet2_utils import grouping_operation

    rng = np.random.default_rng(4)
    f = rng.standard_normal((2, 128, 512)).astype(np.float32)
    idx = rng.integers(0, 512, (2, 128, 16)).astype(np.int32)
    ft = T(f, dev).requires_grad_(True)
    out = grouping_operation(ft, T(idx, dev))
    np.testing.assert_array_equal(out.detach().cpu().numpy(), O.grouping_operation(f, idx))
    go = rng.standard_normal(out.shape).astype(np.float32)
    out.backward(T(go, dev))
    # float atomics: order-dependent rounding only
    np.testing.assert_allclose(ft.grad.cpu().numpy(), O.grouping_operation_grad(go, idx, 512), rtol=1e-5, atol=1e-5)


def test_ball_query_bitexact(dev):
    from svdformer_pointsea_amd.pointnet2_utils import ball_query

    rng = np.random.default_rng(5)
    xyz = rng.random((2, 1024, 3)).astype(np.float32)
    new = xyz[:, ::8].copy()
    new[:, :4] += 5.0  # no neighbours -> zeros
    for r, ns in [(0.1, 16), (0.2, 32), (0.05, 8)]:
        got = ball_query(r, ns, T(xyz, dev), T(new, dev)).cpu().numpy()
        np.testing.assert_array_equal(got, O.ball_query(r, ns, xyz, new))


def test_three_nn_and_interpolate(dev):
    from svdformer_pointsea_amd.pointnet2_utils import three_interpolate, three_nn

    rng = np.random.default_rng(6)
    unknown = rng.random((2, 2048, 3)).astype(np.float32)
    known = rng.random((2, 512, 3)).astype(np.float32)
    dist, idx = three_nn(T(unknown, dev), T(known, dev))
    odist, oidx, _ = O.three_nn(unknown, known)
    np.testing.assert_array_equal(idx.cpu().numpy(), oidx)
    np.testing.assert_array_equal(dist.cpu().numpy(), odist)
    w = rng.random((2, 2048, 3)).astype(np.float32)
    f = rng.standard_normal((2, 32, 512)).astype(np.float32)
    ft = T(f, dev).requires_grad_(True)
    out = three_interpolate(ft, idx, T(w, dev))
    np.testing.assert_array_equal(out.detach().cpu().numpy(), O.three_interpolate(f, oidx, w))
    go = rng.standard_normal(out.shape).astype(np.float32)
    out.backward(T(go, dev))
    np.testing.assert_allclose(ft.grad.cpu().numpy(), O.three_interpolate_grad(go, oidx, w, 512), rtol=1e-5,
                               atol=1e-5)


def test_three_nn_dist_not_differentiable(dev):
    """The reference marks the RETURNED dist (and idx) non-differentiable (pointnet2_utils.py:124-127):
    with a grad-requiring input neither output requires grad."""
    from svdformer_pointsea_amd.pointnet2_utils import three_nn

    rng = np.random.default_rng(7)
    u = T(rng.random((1, 64, 3)).astype(np.float32), dev).requires_grad_(True)
    k = T(rng.random((1, 16, 3)).astype(np.float32), dev).requires_grad_(True)
    dist, idx = three_nn(u, k)
    assert not dist.requires_grad and not idx.requires_grad


# ------------------------------------------------------------------ Chamfer
@pytest.mark.parametrize("name", ["c1", "unit", "tiled"])
def test_chamfer_golden(dev, name):
    from svdformer_pointsea_amd.chamfer3D import chamfer_3DDist

    g = golden("chamfer.npz")
    a, b = g[name + "_a"], g[name + "_b"]
    d1, d2, i1, i2 = [t.cpu().numpy() for t in chamfer_3DDist()(T(a, dev), T(b, dev))]
    # the reference's own test criteria (metrics/CD/unit_test.py:22-33)
    assert ((d1 - g[name + "_d1"]) ** 2).mean() + ((d2 - g[name + "_d2"]) ** 2).mean() < 1e-8
    np.testing.assert_array_equal(i1, g[name + "_i1"])
    np.testing.assert_array_equal(i2, g[name + "_i2"])
    # and bit-exact against the fp32 restatement of chamfer3D.cu
    od1, od2, oi1, oi2 = O.chamfer_forward(a, b)
    np.testing.assert_array_equal(d1, od1)
    np.testing.assert_array_equal(d2, od2)
    np.testing.assert_array_equal(i1, oi1)
    np.testing.assert_array_equal(i2, oi2)


@pytest.mark.parametrize("B,N,M", [(2, 256, 256), (3, 512, 2048), (2, 2048, 2048), (1, 5000, 3001), (2, 1, 7)])
def test_chamfer_bitexact_and_backward(dev, B, N, M):
    from svdformer_pointsea_amd.chamfer3D import chamfer_3DDist

    rng = np.random.default_rng(N + M)
    a = (rng.random((B, N, 3)) - 0.5).astype(np.float32)
    b = (rng.random((B, M, 3)) - 0.5).astype(np.float32)
    at, bt = T(a, dev).requires_grad_(True), T(b, dev).requires_grad_(True)
    d1, d2, i1, i2 = chamfer_3DDist()(at, bt)
    od1, od2, oi1, oi2 = O.chamfer_forward(a, b)
    np.testing.assert_array_equal(d1.detach().cpu().numpy(), od1)
    np.testing.assert_array_equal(d2.detach().cpu().numpy(), od2)
    np.testing.assert_array_equal(i1.cpu().numpy(), oi1)
    np.testing.assert_array_equal(i2.cpu().numpy(), oi2)
    w1 = rng.random((B, N)).astype(np.float32)
    w2 = rng.random((B, M)).astype(np.float32)
    ((d1 * T(w1, dev)).sum() + (d2 * T(w2, dev)).sum()).backward()
    g1, g2 = O.chamfer_backward(a, b, w1, w2, oi1, oi2)
    np.testing.assert_allclose(at.grad.cpu().numpy(), g1, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(bt.grad.cpu().numpy(), g2, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("case", ["loss16384", "hub", "tiled", "inf_grad"])
def test_chamfer_backward_deterministic(dev, case):
    """The one-launch backward (partner terms summed per target in 64-bit fixed point):
    bitwise identical across runs, within fp32 rounding of the oracle's sequential sums
    (chamfer3D.cu:155-195), at the loss's 16384 x 16384 shape, with every source mapped
    to one target (a hub: the fixed-point range at its widest), exact ties, and
    non-finite upstream gradients (fp32 fallback: inf / NaN as the oracle)."""
    from svdformer_pointsea_amd.chamfer3D import chamfer_3DDist

    rng = np.random.default_rng(len(case))
    if case == "loss16384":
        a, b = [(rng.random((2, 16384, 3)) - 0.5).astype(np.float32) for _ in range(2)]
    elif case == "hub":
        a = (rng.random((2, 3000, 3)) - 0.5).astype(np.float32)
        b = (rng.random((2, 2500, 3)) * 100 + 50).astype(np.float32)
        b[:, 17] = 0.0                      # every point of a has b[17] as its nearest
    elif case == "tiled":
        a, b = _tiled(rng, 2, 300, 3000), _tiled(rng, 2, 200, 4100)
    else:
        a, b = [(rng.random((1, n, 3)) - 0.5).astype(np.float32) for n in (2100, 2300)]
    w1 = rng.random(a.shape[:2]).astype(np.float32)
    w2 = rng.random(b.shape[:2]).astype(np.float32)
    if case == "inf_grad":
        w1[0, 3] = np.inf
        w2[0, 11] = np.nan
    grads = []
    for _ in range(2):
        at, bt = T(a, dev).requires_grad_(True), T(b, dev).requires_grad_(True)
        d1, d2, i1, i2 = chamfer_3DDist()(at, bt)
        ((d1 * T(w1, dev)).sum() + (d2 * T(w2, dev)).sum()).backward()
        grads.append((at.grad.cpu().numpy(), bt.grad.cpu().numpy()))
    for x, y in zip(grads[0], grads[1]):
        assert np.array_equal(x, y, equal_nan=True)
    i1, i2 = i1.cpu().numpy(), i2.cpu().numpy()
    g1, g2 = O.chamfer_backward(a, b, w1, w2, i1, i2)
    r1, r2 = _chamfer_grad64(a, b, w1, w2, i1, i2)
    for got, ora, ref in ((grads[0][0], g1, r1), (grads[0][1], g2, r2)):
        fin = np.isfinite(ref)
        assert np.array_equal(np.isnan(got), np.isnan(ref)) and np.array_equal(got[np.isinf(ref)], ref[np.isinf(ref)])
        scale = np.abs(ref[fin]).max()
        # the fp32 rounding of the exact sum (fixed-point partner sums), against float64 ...
        np.testing.assert_allclose(got[fin], ref[fin], rtol=2.5e-7, atol=1e-9 * scale)
        # ... and the oracle's sequential fp32 sums within their own rounding (not for the hub's 3000-term sum)
        if case != "hub":
            np.testing.assert_allclose(got[fin], ora[fin], rtol=1e-5, atol=1e-6 * scale)


@pytest.mark.parametrize("B,N,M,kind", [(2, 512, 600, "gauss"), (3, 2048, 2048, "gauss"), (2, 700, 900, "dup"),
                                        (2, 16384, 16384, "gauss"), (4, 2048, 16384, "gauss")])
def test_sqrt_mean_loss_fused_bitwise(dev, monkeypatch, B, N, M, kind):
    """chamfer_sqrt / chamfer_single_side_sqrt / get_loss as one autograd node (the distance
    gradient formed in one launch, pcops_chamfer_sqrt_mean_grad) against the autograd chain
    (PCOPS_LOSS_FUSED=0): loss values and both clouds' gradients bitwise equal, including
    coincident points (sqrt(d) = 0: an infinite distance gradient either way) and the culled
    search's sizes."""
    from svdformer_pointsea_amd import metrics

    g = torch.Generator().manual_seed(B * N + M)
    a = torch.randn(B, N, 3, generator=g) * 0.45
    b = torch.randn(B, M, 3, generator=g) * 0.45
    if kind == "dup":
        b[:, :N // 2] = a[:, :N // 2]    # half of a's points have an exact partner
    res = {}
    for fused in ("0", "1"):
        monkeypatch.setenv("PCOPS_LOSS_FUSED", fused)
        out = []
        for fn in (metrics.chamfer_sqrt, metrics.chamfer_single_side_sqrt):
            x, y = a.to(dev).requires_grad_(True), b.to(dev).requires_grad_(True)
            loss = fn(x, y)
            gx, gy = torch.autograd.grad(loss * 3.0, (x, y))
            out += [loss.detach(), gx, gy]
        x, y, z = (b[:, :N // 4].to(dev).contiguous().requires_grad_(True),
                   b[:, :N // 2].to(dev).contiguous().requires_grad_(True), b.to(dev).requires_grad_(True))
        gt = a.to(dev)
        loss, parts = metrics.get_loss([x, y, z], gt, sqrt=True, alpha1=1, alpha2=0.5)
        out += [loss.detach(), *[p.detach() for p in parts], *torch.autograd.grad(loss, (x, y, z))]
        res[fused] = out
    for u, v in zip(res["0"], res["1"]):
        torch.testing.assert_close(u, v, rtol=0, atol=0, equal_nan=True)


def test_chamfer_backward_outlier_block_bound(dev):
    """one large partner term sets the fixed-point scale of every target in
    its block, so a target with small terms gets absolute, not relative, resolution.
    The per-target bound is n_j * 2^(e + lg - 63) (n_j partner terms, every finite
    |c| of the block < 2^e, NA < 2^lg sources) plus the final fp32 rounding; checked
    against the float64 sum of the same fp32 terms, target by target, with a 1e6
    upstream gradient on one far source next to O(1) ones."""
    from svdformer_pointsea_amd.chamfer3D import chamfer_3DDist

    rng = np.random.default_rng(77)
    a = (rng.random((1, 2100, 3)) - 0.5).astype(np.float32)
    b = (rng.random((1, 1900, 3)) - 0.5).astype(np.float32)
    a[0, 5] = (60.0, -40.0, 25.0)          # far source: its partner term is ~1e8
    w1 = rng.random(a.shape[:2]).astype(np.float32)
    w2 = rng.random(b.shape[:2]).astype(np.float32)
    w1[0, 5] = 1e6
    at, bt = T(a, dev).requires_grad_(True), T(b, dev).requires_grad_(True)
    d1, d2, i1, i2 = chamfer_3DDist()(at, bt)
    ((d1 * T(w1, dev)).sum() + (d2 * T(w2, dev)).sum()).backward()
    i1, i2 = i1.cpu().numpy(), i2.cpu().numpy()
    r1, r2 = _chamfer_grad64(a, b, w1, w2, i1, i2)
    for got, ref, S, Tc, gS, iS in ((at.grad.cpu().numpy(), r1, b, a, w2, i2),
                                     (bt.grad.cpu().numpy(), r2, a, b, w1, i1)):
        c = (2 * gS[..., None]).astype(np.float32) * (S - np.take_along_axis(Tc, iS[..., None].astype(np.int64), 1))
        e = int(np.frexp(np.abs(c).max())[1])                 # every |c| < 2^e
        lg = int(S.shape[1]).bit_length()                     # NA < 2^lg
        n = np.bincount(iS[0].astype(np.int64), minlength=Tc.shape[1])[None, :, None]
        tol = n * 2.0 ** (e + lg - 63) + 2.0 ** -24 * np.abs(ref) + 1e-30
        err = np.abs(got.astype(np.float64) - ref)
        assert (err <= tol).all(), float((err / tol).max())


def _chamfer_grad64(a, b, w1, w2, i1, i2):
    """Float64 sums of the fp32 terms of chamfer3D.cu:155-174 (own + partners)."""
    out = []
    for S, T, gS, gT, iS, iT in ((b, a, w2, w1, i2, i1), (a, b, w1, w2, i1, i2)):
        # targets = cloud T; own term from T's NN in S, partner terms from S's NN in T
        B = T.shape[0]
        own = (2 * gT[..., None]).astype(np.float32) * (T - np.take_along_axis(S, iT[..., None].astype(np.int64), 1))
        c = (2 * gS[..., None]).astype(np.float32) * (S - np.take_along_axis(T, iS[..., None].astype(np.int64), 1))
        with np.errstate(invalid="ignore"):
            part = np.zeros(T.shape, np.float64)
            for bb in range(B):
                np.add.at(part[bb], iS[bb].astype(np.int64), c[bb].astype(np.float64))
            out.append(own.astype(np.float64) - part)
    return out


def _screen_clouds(kind, rng):
    if kind == "uniform":
        return [(rng.random((2, n, 3)) - 0.5).astype(np.float32) for n in (3000, 5000)]
    if kind == "tiled":  # every point repeated across many sub-tiles: exact ties, slot overflow
        return [_tiled(rng, 2, 300, 3000), _tiled(rng, 2, 200, 4100)]
    if kind == "outliers":  # a few far points inflate the rounding margin
        a, b = [(rng.random((2, n, 3)) - 0.5).astype(np.float32) for n in (2500, 4000)]
        b[:, ::997] *= 1000.0
        a[:, ::501] *= 300.0
        return [a, b]
    if kind == "offset":  # tiny cloud far from the origin: margin >> neighbour gaps
        a, b = [(100.0 + 1e-3 * rng.standard_normal((2, n, 3))).astype(np.float32) for n in (2048, 3000)]
        return [a, b]
    if kind == "nonfinite":
        a, b = [(rng.random((1, n, 3)) - 0.5).astype(np.float32) for n in (2100, 2300)]
        a[0, 5] = np.nan
        b[0, 7] = np.nan
        b[0, 9] = np.inf
        return [a, b]
    raise ValueError(kind)


@pytest.mark.parametrize("q", ["1", "2", "4", "mfma"])
@pytest.mark.parametrize("kind", ["uniform", "tiled", "outliers", "offset", "nonfinite"])
def test_chamfer_screen_bitexact(dev, monkeypatch, kind, q):
    """The screened kernels (e = |t|^2 - 2a.t ranks sub-tiles, the reference
    expression re-derives the winner) forced onto small clouds through
    PCOPS_CHAMFER_Q (VALU screen) / PCOPS_CHAMFER_MFMA=2 (the opt-in fp32-MFMA screen):
    bit-exact distances and indices against the oracle on exact ties, far outliers, a
    cloud far from the origin and non-finite points."""
    from svdformer_pointsea_amd.chamfer3D import chamfer_3DDist

    if q == "mfma":
        monkeypatch.setenv("PCOPS_CHAMFER_MFMA", "2")
    else:
        monkeypatch.setenv("PCOPS_CHAMFER_Q", q)
    a, b = _screen_clouds(kind, np.random.default_rng(len(kind) * 7 + (9 if q == "mfma" else int(q))))
    got = [t.cpu().numpy() for t in chamfer_3DDist()(T(a, dev), T(b, dev))]
    ref = O.chamfer_forward(a, b)
    for x, y in zip(got, ref):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("kernel", [{}, {"PCOPS_CHAMFER_Q": "2"}, {"PCOPS_CHAMFER_Q": "4"},
                                    {"PCOPS_CHAMFER_SCREEN": "0"}, {"PCOPS_CHAMFER_MFMA": "1"},
                                    {"PCOPS_CHAMFER_Q": "4", "PCOPS_CHAMFER_MFMA": "2"}])
def test_chamfer_nonfinite_scan_order(dev, monkeypatch, kernel):
    """The reference's chunked scan order on non-finite data (chamfer3D.cu:16-129), every
    forward kernel (MFMA screen, VALU screen Q=2/4, direct) against the oracle, bitwise: a NaN
    coordinate on a chunk-start target (index 512c) pins (NaN, 0) for c = 0 and hides chunk c
    otherwise; NaN off a chunk start, inf targets and non-finite queries."""
    from svdformer_pointsea_amd.chamfer3D import chamfer_3DDist

    for k, v in kernel.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(23)
    B, N, M = 4, 1100, 1600
    a = (rng.random((B, N, 3)) - 0.5).astype(np.float32)
    b = (rng.random((B, M, 3)) - 0.5).astype(np.float32)
    b[0, 0, 1] = np.nan
    a[0, 1024, 0] = np.nan
    b[1, 512, 0] = np.nan
    b[1, 1024, 2] = np.inf
    a[1, 0, 2] = np.nan
    b[2, 513] = np.nan
    b[2, 0, 0] = np.inf
    a[2, 3] = [np.inf, 0.0, 0.0]
    a[3, 5, 1] = np.nan
    b[3, 1536, 1] = np.nan
    got = [t.cpu().numpy() for t in chamfer_3DDist()(T(a, dev), T(b, dev))]
    ref = O.chamfer_forward(a, b)
    for x, y in zip(got, ref):
        np.testing.assert_array_equal(x, y)
    assert np.isnan(got[0][0]).all() and np.isnan(got[1][1]).all()


def test_chamfer_full_size_one_cloud_bitexact(dev):
    """16384 x 16384 (the loss Chamfer, screened kernel) on one cloud, both directions, vs the oracle."""
    from svdformer_pointsea_amd.chamfer3D import chamfer_3DDist

    g = torch.Generator(device="cpu").manual_seed(11)
    a = (torch.randn(1, 16384, 3, generator=g) * 0.45).numpy()
    b = (torch.randn(1, 16384, 3, generator=g) * 0.45).numpy()
    got = [t.cpu().numpy() for t in chamfer_3DDist()(T(a, dev), T(b, dev))]
    for x, y in zip(got, O.chamfer_forward(a, b)):
        np.testing.assert_array_equal(x, y)


def test_chamfer_full_size_properties(dev):
    """B=32, 16384 x 16384 (the loss Chamfer): symmetry and spot checks."""
    from svdformer_pointsea_amd.chamfer3D import chamfer_3DDist

    g = torch.Generator(device="cpu").manual_seed(7)
    a = (torch.randn(32, 16384, 3, generator=g) * 0.45).to(dev)
    b = (torch.randn(32, 16384, 3, generator=g) * 0.45).to(dev)
    d1, d2, i1, i2 = chamfer_3DDist()(a, b)
    e2, e1, j2, j1 = chamfer_3DDist()(b, a)
    assert torch.equal(d1, e1) and torch.equal(d2, e2) and torch.equal(i1, j1) and torch.equal(i2, j2)
    # the reported distance is the distance to the reported index
    nb = torch.gather(b, 1, i1.long().unsqueeze(-1).expand(-1, -1, 3))
    torch.testing.assert_close(d1, ((a - nb) ** 2).sum(-1), rtol=1e-5, atol=1e-7)
    for bb in (0, 17):
        od1, od2, oi1, oi2 = O.chamfer_forward(a[bb:bb + 1, :2048].cpu().numpy(), b[bb:bb + 1].cpu().numpy())
        s1, s2, si1, si2 = chamfer_3DDist()(a[bb:bb + 1, :2048].contiguous(), b[bb:bb + 1].contiguous())
        np.testing.assert_array_equal(si1.cpu().numpy(), oi1)
        np.testing.assert_array_equal(s1.cpu().numpy(), od1)


# ------------------------------------------------------------------ kNN
def test_knn_golden_bitexact(dev):
    from svdformer_pointsea_amd.model_utils import query_knn, query_knn_point

    k = golden("knn.npz")
    got = query_knn(16, T(k["qk_xyz"], dev), T(k["qk_new"], dev)).cpu().numpy()
    np.testing.assert_array_equal(got, k["qk_idx"])
    got = query_knn(16, T(k["qk_xyz"], dev), T(k["qk_new"], dev), include_self=False).cpu().numpy()
    np.testing.assert_array_equal(got, k["qk_idx_noself"])
    for name, K in [("kp3", 16), ("kp64", 8), ("kp256", 4)]:
        x = T(k[name + "_x"], dev)
        got = query_knn_point(K, x, x)
        assert got.dtype == torch.int64
        np.testing.assert_array_equal(got.cpu().numpy(), k[name + "_idx"])


def test_knn_ties_bitexact_vs_oracle(dev):
    from svdformer_pointsea_amd.model_utils import _knn

    k = golden("knn.npz")
    idx, d = _knn(T(k["qkt_new"], dev), T(k["qkt_xyz"], dev), 16, want_dist=True)
    oidx, od = O.knn(k["qkt_new"], k["qkt_xyz"], 16, return_dist=True)
    np.testing.assert_array_equal(idx.cpu().numpy(), oidx)
    np.testing.assert_array_equal(d.cpu().numpy(), od)
    # reference argsort leaves exact ties unordered: the distances per rank agree
    full = O.square_distance(k["qkt_new"], k["qkt_xyz"])
    np.testing.assert_array_equal(np.take_along_axis(full, k["qkt_idx"].astype(np.int64), -1), od)


def test_group_local_golden(dev):
    from svdformer_pointsea_amd.model_utils import group_local

    k = golden("knn.npz")
    x = T(k["kp3_x"], dev).transpose(1, 2).contiguous()
    g, idx = group_local(x, k=16, return_idx=True)
    np.testing.assert_array_equal(idx.cpu().numpy(), k["gl_idx"])
    np.testing.assert_array_equal(g.cpu().numpy(), k["gl_group"])


@pytest.mark.parametrize("C,N,K,pad", [(3, 2048, 16, 0), (64, 512, 8, 0), (256, 512, 4, 0), (3, 777, 20, 1),
                                       (40, 300, 5, 2), (128, 1024, 16, 0)])
def test_knn_bitexact_vs_oracle(dev, C, N, K, pad):
    from svdformer_pointsea_amd.model_utils import _knn

    rng = np.random.default_rng(C * N + K)
    p = rng.standard_normal((2, N, C)).astype(np.float32)
    q = p[:, : min(N, 300)].copy()
    idx, d = _knn(T(q, dev), T(p, dev), K, pad, want_dist=True)
    oidx, od = O.knn(q, p, K, pad, return_dist=True)
    np.testing.assert_array_equal(idx.cpu().numpy(), oidx)
    np.testing.assert_array_equal(d.cpu().numpy(), od)


def test_fps_subsample_and_sample_and_group(dev):
    from svdformer_pointsea_amd.model_utils import fps_subsample, sample_and_group_knn

    rng = np.random.default_rng(8)
    x = (rng.random((2, 2048, 3)) - 0.5).astype(np.float32)
    sub = fps_subsample(T(x, dev), 512).cpu().numpy()
    oidx = O.furthest_point_sample(x, 512)
    np.testing.assert_array_equal(sub, np.take_along_axis(x, oidx[..., None].astype(np.int64), 1))
    xyz = T(x, dev).transpose(1, 2).contiguous()
    new_xyz, new_points, idx, grouped = sample_and_group_knn(xyz, xyz, 512, 16)
    oknn = O.knn(sub, x, 16)
    np.testing.assert_array_equal(idx.cpu().numpy(), oknn)
    og = O.grouping_operation(x.transpose(0, 2, 1), oknn) - sub.transpose(0, 2, 1)[..., None]
    np.testing.assert_array_equal(grouped.cpu().numpy(), og)
    assert new_points.shape == (2, 6, 512, 16)


def test_errors_are_raised_not_exit(dev):
    from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample, gather_operation

    with pytest.raises(RuntimeError, match="CUDA tensor"):
        furthest_point_sample(torch.zeros(1, 10, 3), 4)
    with pytest.raises(RuntimeError, match="int tensor"):
        gather_operation(torch.zeros(1, 3, 10, device=dev), torch.zeros(1, 4, dtype=torch.int64, device=dev))
    with pytest.raises(RuntimeError, match="contiguous"):
        furthest_point_sample(torch.zeros(1, 3, 10, device=dev).transpose(1, 2), 4)


# ------------------------------------------------------------------ renderers
def test_pcviews_depth_golden(dev):
    from svdformer_pointsea_amd.render import PCViews

    g = golden("depth.npz")
    view = PCViews(TRANS=-0.7, RESOLUTION=224)
    np.testing.assert_array_equal(view.rot_mat.numpy(), g["rot"])
    img = view.get_img(T(g["points"], dev)).cpu().numpy()
    # same pixels as the reference; values equal up to float-atomic summation order
    np.testing.assert_array_equal(img != 0, g["img"] != 0)
    np.testing.assert_allclose(img, g["img"], rtol=1e-6, atol=1e-7)


def test_pcviews_depth_vs_oracle_full_batch(dev):
    from svdformer_pointsea_amd.render import PCViews

    rng = np.random.default_rng(21)
    pts = (rng.random((32, 2048, 3)) - 0.5).astype(np.float32)
    pts[:, ::97] = 0.0
    view = PCViews(TRANS=-0.7, RESOLUTION=224)
    img = view.get_img(T(pts, dev)).cpu().numpy()
    ref = O.points2depth(pts, view.rot_mat.numpy(), view.translation.numpy())
    np.testing.assert_array_equal(img != 0, ref != 0)
    np.testing.assert_allclose(img, ref, rtol=1e-6, atol=1e-7)


def test_pcviews_real_golden(dev):
    from svdformer_pointsea_amd.render import PCViews_Real

    g = golden("grid.npz")
    real = PCViews_Real(TRANS=-0.7)
    np.testing.assert_array_equal(real.rot_mat.numpy(), g["rot"])
    np.testing.assert_array_equal(real.rot_mat2.numpy(), g["rot2"])
    np.testing.assert_allclose(real.kernel.numpy(), g["kern"], rtol=0, atol=0)
    grid = real.points2grid(T(g["points"], dev)).cpu().numpy()
    np.testing.assert_array_equal(grid, g["grid"])
    img = real.get_img(T(g["points"], dev)).cpu().numpy()
    np.testing.assert_allclose(img[:, 0], g["img0"], atol=1e-6)
    np.testing.assert_array_equal(img[:, 0], img[:, 2])


@pytest.mark.parametrize("dtype,K,C", [(torch.float32, 16, 128), (torch.float32, 16, 256), (torch.bfloat16, 16, 128),
                                       (torch.bfloat16, 16, 256), (torch.float32, 4, 96), (torch.bfloat16, 8, 64),
                                       (torch.float32, 8, 64), (torch.bfloat16, 16, 64)])
def test_pcsa_kernel_matches_torch_chain(dev, dtype, K, C):
    """PCSA (model_utils.py:408-430): the libpcops patch kernel vs the
    reference's permute / DCT matmul / gate / IDCT matmul chain, fwd + bwd."""
    from svdformer_pointsea_amd.svdformer import PCSA

    torch.manual_seed(K + C)
    m = PCSA(C, K).to(dev)
    B, S = 2, 37
    x0 = torch.randn(B, C, S, K, device=dev).to(dtype).contiguous(memory_format=torch.channels_last)
    go = torch.randn(B, C, S, K, device=dev).to(dtype)
    amp = dtype == torch.bfloat16  # bf16 features only occur under autocast
    xa = x0.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        ya = m(xa)                                 # kernel path (channels_last input)
    (ya.float() * go.float()).sum().backward()
    ga = [p.grad.clone() for p in m.parameters()]
    m.zero_grad()
    xb = x0.contiguous().clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        yb = m(xb)                                 # reference chain (NCHW input)
    (yb.float() * go.float()).sum().backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 2e-5
    torch.testing.assert_close(ya.float(), yb.float(), rtol=tol, atol=tol)
    torch.testing.assert_close(xa.grad.float(), xb.grad.float(), rtol=tol, atol=tol)
    for a, b in zip(ga, (p.grad for p in m.parameters())):
        torch.testing.assert_close(a.float(), b.float(), rtol=tol * 5, atol=tol * 5)


@pytest.mark.parametrize("dtype,K,C", [(torch.bfloat16, 16, 128), (torch.float32, 8, 64)])
def test_pcsa_channel_mean_broadcast_grad_bitwise(dev, monkeypatch, dtype, K, C):
    """PCSA's gate input x.mean(dim=1) through _ChannelMean (the backward hands autograd the
    broadcast gradient as an expanded view of grad / C) against torch's MeanBackward, which
    materialises it: output, input gradient and parameter gradients bitwise equal."""
    import svdformer_pointsea_amd.svdformer as SV

    torch.manual_seed(K * C)
    m = SV.PCSA(C, K).to(dev)
    B, S = 3, 41
    x0 = torch.randn(B, C, S, K, device=dev).to(dtype).contiguous(memory_format=torch.channels_last)
    go = torch.randn(B, C, S, K, device=dev).to(dtype).contiguous(memory_format=torch.channels_last)
    amp = dtype == torch.bfloat16
    res = {}
    for on in (False, True):
        monkeypatch.setattr(SV, "_CHANNEL_MEAN", on)
        m.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            y = m(x)
        y.backward(go.to(y.dtype))
        res[on] = [y.detach(), x.grad] + [p.grad for p in m.parameters()]
    for u, v in zip(res[False], res[True]):
        assert torch.equal(u, v), (u.float() - v.float()).abs().max().item()


@pytest.mark.parametrize("B,S,N,C,K,pad,kind", [(32, 512, 512, 64, 8, 0, "rand"), (16, 1024, 1024, 256, 4, 0, "rand"),
                                                 (16, 1024, 1024, 64, 8, 0, "tiled"), (2, 300, 300, 40, 5, 2, "rand"),
                                                 (3, 200, 777, 128, 20, 1, "tiled"), (2, 1000, 100, 32, 16, 0, "rand"),
                                                 (1, 64, 4000, 96, 32, 0, "rand")])
def test_knn_feature_split_bitexact(dev, monkeypatch, B, S, N, C, K, pad, kind):
    """The streamed, candidate-split feature-space kNN (knnC3_kernel + knn_merge_kernel) against
    knnC2_kernel (pcops_knn): idx and dist bitwise at the model shapes (PCN gcn_2, PointSea
    gcn_2 / gcn_3), with exact ties (duplicated rows), pad, more queries than candidates, and
    empty trailing splits; the oracle on the small cases."""
    import svdformer_pointsea_amd.model_utils as MU

    rng = np.random.default_rng(B * S + N + C)
    if kind == "tiled":
        u = rng.standard_normal((B, max(8, N // 5), C)).astype(np.float32)
        p = u[:, rng.integers(0, u.shape[1], N)]
    else:
        p = rng.standard_normal((B, N, C)).astype(np.float32)
    q = p[:, :S].copy() if S <= N else rng.standard_normal((B, S, C)).astype(np.float32)
    pt = T(p, dev)
    qt = pt if S == N else T(q, dev)
    got = MU._knn(qt, pt, K, pad, want_dist=True)
    monkeypatch.setattr(MU, "_KNN_SORTED", False)
    ref = MU._knn(qt, pt, K, pad, want_dist=True)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    if B * S * N <= 4_000_000:
        oidx, od = O.knn(q, p, K, pad, return_dist=True)
        np.testing.assert_array_equal(got[0].cpu().numpy(), oidx)
        np.testing.assert_array_equal(got[1].cpu().numpy(), od)


@pytest.mark.parametrize("B,S,N,K,pad,kind", [(32, 2048, 2048, 16, 0, "surface"), (32, 512, 2048, 16, 0, "fps"),
                                              (4, 1024, 1024, 16, 1, "tiled"), (3, 333, 1500, 8, 1, "cluster"),
                                              (2, 700, 700, 20, 0, "flat"), (2, 300, 300, 16, 0, "nan"),
                                              (2, 100, 17, 16, 1, "surface"), (2, 256, 4096, 32, 0, "far"),
                                              (1, 2000, 64, 4, 0, "line"), (8, 640, 640, 16, 0, "zero")])
def test_knn3_adversarial_bitexact(dev, monkeypatch, B, S, N, K, pad, kind):
    """C = 3 kNN (knn3_kernel: batched candidate reads, cross-wave threshold sharing) through both
    entry points against the oracle: idx and dist bitwise.  Clouds that stress the shared
    thresholds: exact duplicates (ties at a threshold), tight clusters far apart, a flat cloud,
    NaN points, N = K + pad, queries far outside the candidates' box, points on a line, an
    all-zero cloud."""
    import svdformer_pointsea_amd.model_utils as MU

    rng = np.random.default_rng(B * S + N + K)
    if kind in ("surface", "fps", "nan", "far"):
        v = rng.standard_normal((B, N, 3)).astype(np.float32)
        p = (v / np.linalg.norm(v, axis=-1, keepdims=True)).astype(np.float32)
    elif kind == "tiled":
        u = rng.random((B, N // 8, 3), dtype=np.float32)
        p = u[:, rng.integers(0, u.shape[1], N)]
    elif kind == "cluster":
        c = rng.standard_normal((B, 5, 3)).astype(np.float32) * 10
        p = (c[:, rng.integers(0, 5, N)] + 1e-3 * rng.standard_normal((B, N, 3))).astype(np.float32)
    elif kind == "flat":
        p = rng.random((B, N, 3), dtype=np.float32)
        p[..., 2] = 0.5
    elif kind == "line":
        t = rng.random((B, N, 1), dtype=np.float32)
        p = (t * np.array([1.0, 2.0, -0.5], np.float32)).astype(np.float32)
    else:
        p = np.zeros((B, N, 3), np.float32)
    if kind == "nan":
        p[:, ::37] = np.nan
    p = np.ascontiguousarray(p)
    if kind == "fps":
        q = p[:, rng.permutation(N)[:S]].copy()
    elif kind == "far":
        q = (rng.standard_normal((B, S, 3)) * 50).astype(np.float32)
    elif S <= N:
        q = p[:, :S].copy()
    else:
        q = rng.random((B, S, 3), dtype=np.float32)
    pt = T(p, dev)
    qt = pt if (S == N and kind not in ("fps", "far")) else T(q, dev)
    got = MU._knn(qt, pt, K, pad, want_dist=True)
    monkeypatch.setattr(MU, "_KNN_SORTED", False)
    ref = MU._knn(qt, pt, K, pad, want_dist=True)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    if B * S * N <= 4_000_000 and kind != "nan":
        oidx, od = O.knn(q, p, K, pad, return_dist=True)
        np.testing.assert_array_equal(got[0].cpu().numpy(), oidx)
        np.testing.assert_array_equal(got[1].cpu().numpy(), od)


@pytest.mark.parametrize("B,N,M,kind", [(2, 16384, 16384, "gauss"), (3, 16384, 8192, "surface"),
                                        (2, 8192, 8192, "dup"), (2, 4096, 16000, "clusters"),
                                        (3, 6000, 5000, "nonfinite"), (2, 4096, 4096, "same"),
                                        (2, 5000, 7000, "huge"), (2, 4096, 6000, "huge2"), (2, 4096, 4100, "tiny"), (3, 1024, 16384, "surface"),
                                        (2, 16384, 2048, "gauss"), (32, 16384, 16384, "pcn")])
@pytest.mark.parametrize("es", ["1", "0"])
def test_chamfer_culled_bitexact(dev, B, N, M, kind, es, monkeypatch):
    """The spatially culled Chamfer search (pcops_chamfer_forward_ws: Morton-sorted clouds, tile
    boxes, waves taking tiles nearest-first and skipping those beyond their queries' bounds under a
    rigorous margin) against the
    all-pairs screens (pcops_chamfer_forward): dist and idx bitwise, both directions.  Exact
    duplicates (ties across tiles), far clusters, NaN / inf points (culling off, the reference's
    first-candidate rule), a single repeated point, coordinates whose squares overflow, and
    coordinates whose distances are denormal."""
    from svdformer_pointsea_amd._lib import Workspace, call, lib, ptr, stream_of

    # pass 1 in both forms: the screen expression (ES=1, the default) and the direct distance
    # (ES=0, chamfer_cull_kernel<false>: its own tie tracking and tile selection); read per call
    monkeypatch.setenv("PCOPS_CHAMFER_CULL_ES", es)
    if es == "0" and kind == "pcn":
        pytest.skip("the B = 32 case runs once, with the default pass 1")
    g = torch.Generator().manual_seed(B * N + M)
    if kind in ("gauss", "pcn"):
        a, b = torch.randn(B, N, 3, generator=g) * 0.45, torch.randn(B, M, 3, generator=g) * 0.45
    elif kind == "surface":
        def surf(n):
            v = torch.randn(B, n, 3, generator=g)
            return v / v.norm(dim=-1, keepdim=True) * torch.tensor([1.0, 0.6, 0.3])
        a, b = surf(N), surf(M)
    elif kind == "dup":
        u = torch.randn(B, 1500, 3, generator=g)
        a = u[:, torch.randint(0, 1500, (N,), generator=g)]
        b = u[:, torch.randint(0, 1500, (M,), generator=g)]
    elif kind == "clusters":
        c = torch.randn(B, 6, 3, generator=g) * 50
        a = c[:, torch.randint(0, 6, (N,), generator=g)] + 1e-2 * torch.randn(B, N, 3, generator=g)
        b = c[:, torch.randint(0, 6, (M,), generator=g)] + 1e-2 * torch.randn(B, M, 3, generator=g)
        a[:, ::997] = 1e4   # far outliers
    elif kind == "nonfinite":
        a, b = torch.randn(B, N, 3, generator=g), torch.randn(B, M, 3, generator=g)
        a[0, 5, 1] = float("nan")
        b[0, 0, 2] = float("inf")       # target 0: inf - inf / inf distances for every query
        b[1, 7, 0] = float("-inf")
        b[1, 1536, 1] = float("nan")    # a chunk-start target: chunk 3 hidden (reference scan order)
        a[2, 0] = float("nan")
    elif kind == "same":
        a = torch.full((B, N, 3), 0.25)
        b = torch.full((B, M, 3), 0.25)
    elif kind == "huge":
        a, b = torch.randn(B, N, 3, generator=g) * 1e19, torch.randn(B, M, 3, generator=g) * 1e19
    elif kind == "huge2":  # |t|^2 and 2 a.t overflow fp32: the screens' e is +-inf / NaN
        a, b = torch.randn(B, N, 3, generator=g) * 4e19, torch.randn(B, M, 3, generator=g) * 4e19
        a[:, ::3] *= 1e-10  # and some queries small enough for finite distances
    else:
        a, b = torch.randn(B, N, 3, generator=g) * 1e-20, torch.randn(B, M, 3, generator=g) * 1e-20
    a, b = a.float().contiguous().to(dev), b.float().contiguous().to(dev)
    outs = []
    for ws_path in (False, True):
        d1, d2 = torch.empty(B, N, device=dev), torch.empty(B, M, device=dev)
        i1 = torch.empty(B, N, dtype=torch.int32, device=dev)
        i2 = torch.empty(B, M, dtype=torch.int32, device=dev)
        if ws_path:
            wsb = lib().pcops_chamfer_workspace_bytes(B, N, M)
            assert wsb > 0
            ws = Workspace.get(a.device, wsb)
            call("cull", lib().pcops_chamfer_forward_ws, ptr(a), ptr(b), B, N, M, ptr(d1), ptr(d2), ptr(i1), ptr(i2),
                 ptr(ws), wsb, stream_of(a))
        else:
            call("screen", lib().pcops_chamfer_forward, ptr(a), ptr(b), B, N, M, ptr(d1), ptr(d2), ptr(i1), ptr(i2),
                 stream_of(a))
        outs.append((d1, d2, i1, i2))
    for x, y in zip(*outs):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
    # and directly against the oracle (chamfer3D.cu:12-134 restated) on every case; at B = 32 on
    # three clouds of the batch (first, middle, last), which keeps the CPU check to seconds
    sel = [0, B // 2, B - 1] if kind == "pcn" else list(range(B))
    ref = O.chamfer_forward(a[sel].cpu().numpy(), b[sel].cpu().numpy())
    for x, y in zip(outs[1], ref):
        np.testing.assert_array_equal(x[sel].cpu().numpy(), y)
