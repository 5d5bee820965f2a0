"""EdgeConv's fused edge features (model_utils.edge_features -> pcops_edge_group /
pcops_edge_group_grad) against the unfused reference composite of
models/model_utils.py:869-877 (group_local -> central.repeat -> central - neigh
-> cat -> channels_last) and against the reference's own group_local golden.

Forward: bitwise.  Backward: the fused gradient against the float64 sum of the
same upstream gradient (own term + index_points scatter), at fp32 tolerance,
or one bf16 rounding when the input is bf16 (PointSea's gcn_3 under autocast).
Shapes: gcn_1 (C = 3, K = 16, N = 2048), gcn_2 (C = 64, K = 8, N = 512),
PointSea's gcn_3 (C = 256, K = 4, N = 1024; models_PointSea/PointSea.py:234-236)."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu

SHAPES = [(4, 3, 2048, 16), (4, 64, 512, 8), (2, 256, 1024, 4), (2, 40, 300, 5)]


def _unfused(x, k):
    """models/model_utils.py:869-877 as the reference writes it (with this package's group_local)."""
    from svdformer_pointsea_amd.model_utils import group_local

    neigh = group_local(x.float(), k=k).contiguous().to(x.dtype)
    central = x.unsqueeze(3).repeat(1, 1, 1, k)
    return torch.cat((central - neigh, central), dim=1).contiguous(memory_format=torch.channels_last)


def _grad_ref(g, idx, C):
    """float64: dx[b,n] = sum_k (g_e + g_c)[b,n,k] - sum_{(m,k): idx[b,m,k] = n} g_e[b,m,k]."""
    g = g.double()                                   # (B, N, K, 2C)
    B, N, K, _ = g.shape
    own = (g[..., :C] + g[..., C:]).sum(2)           # (B, N, C)
    scat = torch.zeros(B, N, C, dtype=torch.float64, device=g.device)
    for b in range(B):
        scat[b].index_add_(0, idx[b].reshape(-1).long(), g[b, :, :, :C].reshape(-1, C))
    return own - scat


@pytest.mark.parametrize("B,C,N,K", SHAPES)
@pytest.mark.parametrize("mode", ["fp32", "fp32->bf16", "bf16"])
def test_edge_features_forward_bitwise_backward_close(dev, B, C, N, K, mode):
    from svdformer_pointsea_amd.model_utils import _knn, edge_features

    gen = torch.Generator().manual_seed(B * 1000 + C * 10 + K)
    x0 = torch.randn(B, C, N, generator=gen).to(dev)
    in_dt = torch.bfloat16 if mode == "bf16" else torch.float32
    out_dt = torch.float32 if mode == "fp32" else torch.bfloat16
    x = x0.to(in_dt).requires_grad_(True)
    got = edge_features(x, K, out_dt)
    assert got.shape == (B, 2 * C, N, K) and got.dtype == out_dt
    assert got.is_contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        ref = _unfused(x.detach(), K).to(out_dt)
    assert torch.equal(got, ref)
    # backward: upstream gradient in the feature's dtype, as the first conv returns it
    g = torch.randn(B, 2 * C, N, K, generator=gen).to(dev).to(out_dt).contiguous(memory_format=torch.channels_last)
    got.backward(g)
    pts = x.detach().float().transpose(1, 2).contiguous()
    idx = _knn(pts, pts, K)
    want = _grad_ref(g.permute(0, 2, 3, 1), idx, C).transpose(1, 2)     # (B, C, N) float64
    gx = x.grad.double()
    scale = want.abs().max().item()
    if in_dt == torch.float32:
        assert (gx - want).abs().max().item() <= 2e-6 * max(scale, 1.0)
    else:   # fp32 accumulation, one rounding to bf16
        assert ((gx - want).abs() <= want.abs() * 2 ** -8 + 1e-6 * scale).all()


def test_edge_features_group_local_golden(dev):
    """The neighbour half equals central minus the reference's own group_local output."""
    from svdformer_pointsea_amd.model_utils import edge_features

    k = golden("knn.npz")
    x = torch.from_numpy(k["kp3_x"]).to(dev).transpose(1, 2).contiguous()   # (2, 3, 1024)
    feat = edge_features(x, 16, torch.float32).cpu().numpy()               # (2, 6, 1024, 16)
    xc = k["kp3_x"].transpose(0, 2, 1)[..., None]                          # (2, 3, 1024, 1)
    np.testing.assert_array_equal(feat[:, :3], xc - k["gl_group"])
    np.testing.assert_array_equal(feat[:, 3:], np.broadcast_to(xc, k["gl_group"].shape))


@pytest.mark.parametrize("cin,cout,k,N", [(3, 64, 16, 2048), (64, 256, 8, 512), (256, 512, 4, 1024)])
def test_edgeconv_module_fused_equals_unfused(dev, cin, cout, k, N):
    """svdformer.EdgeConv (models/model_utils.py:847-881) under bf16 autocast: the fused
    module output is bitwise the unfused one; input / weight gradients agree to bf16 noise."""
    import copy

    from svdformer_pointsea_amd import svdformer as S

    torch.manual_seed(cin)
    m = S.EdgeConv(cin, cout, k).to(dev)
    m2 = copy.deepcopy(m)
    x = torch.randn(2, cin, N, device=dev)
    xs = [x.clone().requires_grad_(cin > 3) for _ in range(2)]
    outs = []
    saved = S._EDGE_FUSED
    try:
        for fused, mod, xi in ((True, m, xs[0]), (False, m2, xs[1])):
            S._EDGE_FUSED = fused
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = mod(xi)
            y.float().square().mean().backward()
            outs.append(y.detach())
    finally:
        S._EDGE_FUSED = saved
    assert torch.equal(outs[0], outs[1])
    for (n, p1), (_, p2) in zip(m.named_parameters(), m2.named_parameters()):
        torch.testing.assert_close(p1.grad, p2.grad, rtol=2e-2, atol=1e-5 * max(1.0, p2.grad.abs().max().item()),
                                   msg=n)
    if cin > 3:
        # same upstream gradient; only the summation order of the edge-feature backward differs
        torch.testing.assert_close(xs[0].grad, xs[1].grad, rtol=1e-4, atol=1e-6 * xs[1].grad.abs().max().item())
