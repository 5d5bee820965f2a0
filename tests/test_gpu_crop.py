"""pcops_crop_pack -- seprate_point_cloud's crop order and packing (utils/helpers.py:96-111) in one launch --
against the torch form it replaces (torch.argsort + data._pack), bitwise: random clouds at the train shape,
non-power-of-two and tiny clouds, tied distances (index order, as torch's stable radix sort), NaN distances
(sorted last), start / count at the edges, and the whole seprate_point_cloud fused vs unfused."""
import pytest
import torch

from svdformer_pointsea_amd import data as D
from svdformer_pointsea_amd._lib import lib, ptr, stream_of

pytestmark = pytest.mark.gpu


def _bits(t):
    return t.contiguous().view(torch.int32)


def _reference(dist, xyz, start, count, n_max):
    order = torch.argsort(dist, dim=-1, descending=False, stable=True)
    N = xyz.shape[1]
    cnt = (N - start) if count is None else count
    return D._pack(xyz, order, start, cnt, n_max), cnt.to(torch.int32)


def _cloud(B, N, seed, kind, dev):
    g = torch.Generator().manual_seed(seed)
    xyz = torch.randn(B, N, 3, generator=g) * 0.45
    if kind == "ties":   # every point four times: equal distances everywhere
        xyz = xyz[:, : max(1, N // 4)].repeat_interleave(4, dim=1)[:, :N]
        if xyz.shape[1] < N:
            xyz = torch.cat([xyz, xyz[:, : N - xyz.shape[1]]], dim=1)
    if kind == "nan":
        xyz[:, ::97, 1] = float("nan")
    c = torch.nn.functional.normalize(torch.randn(B, 1, 3, generator=g), p=2, dim=-1)
    xyz, c = xyz.to(dev), c.to(dev)
    return xyz.contiguous(), torch.norm(c - xyz, p=2, dim=-1)


@pytest.mark.parametrize("B,N,kind", [(16, 8192, "plain"), (4, 2048, "plain"), (3, 3000, "plain"), (2, 1, "plain"),
                                      (2, 5, "plain"), (4, 2048, "ties"), (3, 1000, "nan"), (2, 16384, "plain")])
def test_crop_pack_matches_argsort_pack(dev, B, N, kind):
    xyz, dist = _cloud(B, N, B * 131 + N, kind, dev)
    g = torch.Generator(device=dev).manual_seed(N)
    lo, hi = N // 4, (3 * N) // 4
    num_crop = torch.randint(lo, hi + 1, (B,), device=dev, generator=g)
    cases = [(num_crop, None, N - lo),                          # the input part: ranks num_crop.. (count N - start)
             (torch.zeros_like(num_crop), num_crop, max(1, hi)),  # the crop part: ranks 0 .. num_crop - 1
             (torch.zeros_like(num_crop), None, N),             # everything
             (torch.full_like(num_crop, N), None, 3),            # nothing kept: zero tail only
             (torch.full_like(num_crop, max(0, N - 1)), None, N)]
    for start, count, n_max in cases:
        out, counts = D._crop_pack(dist, xyz, start, count, n_max)
        ref, rc = _reference(dist, xyz, start, count, n_max)
        assert torch.equal(counts, rc), (start, count)
        assert torch.equal(_bits(out), _bits(ref)), (kind, n_max)


def test_crop_pack_rejects(dev):
    xyz = torch.zeros(1, 16385, 3, device=dev)
    dist = torch.zeros(1, 16385, device=dev)
    start = torch.zeros(1, dtype=torch.int64, device=dev)
    out = torch.empty(1, 8, 3, device=dev)
    st = lib().pcops_crop_pack(ptr(dist), ptr(xyz), ptr(start), None, 1, 16385, 8, ptr(out), None, stream_of(xyz))
    assert st != 0
    st = lib().pcops_crop_pack(ptr(dist), ptr(xyz), None, None, 1, 8, 8, ptr(out), None, stream_of(xyz))
    assert st != 0
    assert lib().pcops_crop_pack(None, None, None, None, 0, 8, 8, None, None, stream_of(xyz)) == 0


@pytest.mark.parametrize("want_crop", [True, False])
def test_seprate_point_cloud_fused_bitwise(dev, monkeypatch, want_crop):
    """seprate_point_cloud with the crop on pcops_crop_pack == with torch.argsort + _pack, bitwise, at the
    ShapeNet-55 train shape (B = 16, 8192 points, crop [2048, 6144]) and at 2048 points."""
    from bench import synth_55

    for B, n in ((16, 8192), (4, 2048)):
        _, gt = synth_55(B, 21 + n, dev)
        gt = gt[:, :n].contiguous()
        crop = [n // 4, 3 * n // 4]
        out = []
        for fused in (True, False):
            monkeypatch.setattr(D, "_CROP_FUSED", fused)
            out.append(D.seprate_point_cloud(gt, n, crop, generator=torch.Generator(device=dev).manual_seed(3),
                                             want_crop=want_crop))
        (a, ca), (b, cb) = out
        assert torch.equal(a, b)
        assert (ca is None and cb is None) or torch.equal(ca, cb)
