"""The fused SA-module grouping (pcops_sa_group: FPS -> kNN -> one grouping
launch into the first conv's channels_last input) against the unfused
sample_and_group_knn path of the same module (models/model_utils.py:323-356,
432-487): forward bitwise, gradients to 1e-6 (float atomics in both), fp32 and
bf16 autocast, for the two SVDFormer SA modules' shapes."""
import copy

import numpy as np
import pytest
import torch

import svdformer_pointsea_amd.svdformer as S
import svdformer_pointsea_amd.svdformer as S_mod

pytestmark = pytest.mark.gpu


def _run(mod, xyz, pts, amp, fused, monkeypatch):
    monkeypatch.setattr(S, "_SA_FUSED", fused)
    p = pts.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        new_xyz, new_points, idx = mod(xyz, p)
    g = torch.randn(new_points.shape, generator=torch.Generator().manual_seed(3)).to(new_points.device)
    (new_points.float() * g).sum().backward()
    grads = {n: q.grad.clone() for n, q in mod.named_parameters() if q.grad is not None}
    mod.zero_grad(set_to_none=True)
    return new_xyz, new_points.float().contiguous(), idx, p.grad.clone(), grads


@pytest.mark.parametrize("amp", [False, True])
@pytest.mark.parametrize("stage", [1, 2])
def test_sa_module_fused_equals_unfused(dev, monkeypatch, amp, stage):
    torch.manual_seed(stage)
    B = 4
    if stage == 1:   # sa_module_1: 2048 -> 512, K 16, points = the cloud itself (C = 3)
        mod = S.PointNet_SA_Module_KNN(512, 16, 3, [64, 128], if_bn=False, if_idx=True, use_pcsa=True)
        xyz = (torch.rand(B, 3, 2048) - 0.5).to(dev)
        pts = xyz.clone()
    else:            # sa_module_2: 512 -> 128, K 16, C = 128 features
        mod = S.PointNet_SA_Module_KNN(128, 16, 128, [128, 256], if_bn=False, if_idx=True, use_pcsa=True)
        xyz = (torch.rand(B, 3, 512) - 0.5).to(dev)
        pts = torch.randn(B, 128, 512).to(dev)
    mod = mod.to(dev)
    for m in mod.modules():
        if isinstance(m, torch.nn.Conv2d):
            m.to(memory_format=torch.channels_last)
    ref = _run(copy.deepcopy(mod), xyz, pts, amp, False, monkeypatch)
    got = _run(copy.deepcopy(mod), xyz, pts, amp, True, monkeypatch)
    assert torch.equal(got[0], ref[0]) and torch.equal(got[2], ref[2])
    assert torch.equal(got[1], ref[1])   # same grouped values -> same GEMMs -> same bits
    tol = dict(rtol=2e-2, atol=2e-2) if amp else dict(rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(got[3], ref[3], **tol)
    for n in ref[4]:
        torch.testing.assert_close(got[4][n], ref[4][n], **tol, msg=n)


def test_sa_group_kernel_values(dev):
    """pcops_sa_group itself: xyz[idx] - centre | points_t[idx], including
    out-of-range indices (zero rows, as group_points), bf16 output."""
    from svdformer_pointsea_amd.model_utils import _SAGroup

    rng = np.random.default_rng(0)
    B, N, S_, K, C = 2, 300, 40, 7, 5
    xyz = torch.from_numpy(rng.random((B, N, 3)).astype(np.float32)).to(dev)
    ctr = torch.from_numpy(rng.random((B, S_, 3)).astype(np.float32)).to(dev)
    pts = torch.from_numpy(rng.standard_normal((B, N, C)).astype(np.float32)).to(dev)
    idx = torch.from_numpy(rng.integers(0, N, (B, S_, K)).astype(np.int32)).to(dev)
    idx[0, 0, 0] = N + 3   # out of range -> zeros (then minus the centre for xyz)
    out = _SAGroup.apply(xyz, ctr, pts, idx, torch.float32)
    il = idx.long().clamp(max=N - 1)
    gx = torch.gather(xyz, 1, il.view(B, -1, 1).expand(-1, -1, 3)).view(B, S_, K, 3)
    gp = torch.gather(pts, 1, il.view(B, -1, 1).expand(-1, -1, C)).view(B, S_, K, C)
    gx[0, 0, 0] = 0
    gp[0, 0, 0] = 0
    ref = torch.cat([gx - ctr.unsqueeze(2), gp], -1)
    assert torch.equal(out, ref)
    out16 = _SAGroup.apply(xyz, ctr, pts, idx, torch.bfloat16)
    assert torch.equal(out16, ref.to(torch.bfloat16))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,S,K,C", [(4, 512, 16, 128), (2, 64, 8, 256), (3, 17, 5, 40)])
def test_max_over_neighbours_kernel(dev, dt, B, S, K, C):
    """pcops_max_k / _grad vs torch.max(dim=2) on (B, S, K, C): values bitwise,
    gradient routed to the same (first) maximising k -- with many exact ties
    (small-integer data) and a NaN."""
    g = torch.Generator().manual_seed(K * C)
    x = torch.randint(-4, 5, (B, S, K, C), generator=g).to(dt).to(dev)
    x[0, 0, 2, 3] = float("nan")
    xa = x.clone().requires_grad_(True)
    xb = x.clone().requires_grad_(True)
    out = S_mod._MaxK.apply(xa)
    ref = torch.max(xb, dim=2)[0]
    assert torch.equal(out.isnan(), ref.isnan())
    assert torch.equal(torch.nan_to_num(out), torch.nan_to_num(ref))
    go = torch.randn(out.shape, generator=g).to(dt).to(dev)
    out.backward(go)
    ref.backward(go)
    assert torch.equal(xa.grad, xb.grad)
