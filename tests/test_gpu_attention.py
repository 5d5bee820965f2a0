"""GPU parity of the attention core (fp32 MFMA path: 1e-5 abs, the north-star
tolerance; bf16 path: bf16-appropriate tolerance) and of the reference's
attention blocks against golden vectors from the reference's own modules."""
import math

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SHAPES = [  # (B, H, Lq, Lk, E)
    (2, 4, 3, 3, 256),      # SVFNet viewattn
    (2, 4, 128, 128, 512),  # SVFNet sa (hd 128)
    (1, 8, 512, 512, 768),  # refine1 (hd 96)
    (1, 8, 200, 77, 512),   # ragged cross (hd 64)
    (1, 8, 2048, 512, 512), # refine2 cross
    (2, 2, 70, 130, 64),    # hd 32
]


def _qkv(B, H, Lq, Lk, E, dev, dtype=torch.float32, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    q = torch.randn(Lq, B, E, generator=g)
    k = torch.randn(Lk, B, E, generator=g)
    v = torch.randn(Lk, B, E, generator=g)
    return [t.to(dev, dtype) for t in (q, k, v)]


def _ref(q, k, v, H):
    """float64 math of nn.MultiheadAttention's core on (L,B,E) inputs."""
    Lq, B, E = q.shape
    hd = E // H
    qq = q.double().reshape(Lq, B * H, hd).transpose(0, 1)
    kk = k.double().reshape(-1, B * H, hd).transpose(0, 1)
    vv = v.double().reshape(-1, B * H, hd).transpose(0, 1)
    s = qq @ kk.transpose(1, 2) / math.sqrt(hd)
    o = torch.softmax(s, -1) @ vv
    return o.transpose(0, 1).reshape(Lq, B, E)


@pytest.mark.parametrize("B,H,Lq,Lk,E", SHAPES)
def test_core_forward_fp32(dev, B, H, Lq, Lk, E):
    from svdformer_pointsea_amd.attention import attention_core

    q, k, v = _qkv(B, H, Lq, Lk, E, dev)
    o = attention_core(q, k, v, H)
    ref = _ref(q, k, v, H)
    assert (o.double() - ref).abs().max().item() < 1e-5
    # oracle cross-check on one head
    hd = E // H
    oo = O.attention_core(q[:, 0, :hd].cpu().numpy()[None], k[:, 0, :hd].cpu().numpy()[None],
                          v[:, 0, :hd].cpu().numpy()[None])[0]
    np.testing.assert_allclose(o[:, 0, :hd].cpu().numpy(), oo, atol=1e-5)


@pytest.mark.parametrize("B,H,Lq,Lk,E", SHAPES)
def test_core_backward_fp32(dev, B, H, Lq, Lk, E):
    from svdformer_pointsea_amd.attention import attention_core

    q, k, v = _qkv(B, H, Lq, Lk, E, dev, seed=1)
    g = torch.randn(Lq, B, E, generator=torch.Generator().manual_seed(5)).to(dev)
    qs, ks, vs = [t.clone().requires_grad_(True) for t in (q, k, v)]
    (attention_core(qs, ks, vs, H) * g).sum().backward()
    qd, kd, vd = [t.double().clone().requires_grad_(True) for t in (q, k, v)]
    (_ref(qd, kd, vd, H) * g.double()).sum().backward()
    for a, b in [(qs.grad, qd.grad), (ks.grad, kd.grad), (vs.grad, vd.grad)]:
        err = (a.double() - b).abs().max().item()
        assert err < 1e-4 * max(1.0, b.abs().max().item()), err


@pytest.mark.parametrize("B,H,Lq,Lk,E", SHAPES)
def test_core_bf16(dev, B, H, Lq, Lk, E):
    from svdformer_pointsea_amd.attention import attention_core

    q, k, v = _qkv(B, H, Lq, Lk, E, dev, seed=2)
    qb, kb, vb = [t.to(torch.bfloat16).requires_grad_(True) for t in (q, k, v)]
    o = attention_core(qb, kb, vb, H)
    assert o.dtype == torch.bfloat16
    ref = _ref(qb.detach().float(), kb.detach().float(), vb.detach().float(), H)
    assert (o.double() - ref).abs().max().item() < 3e-2
    g = torch.randn(Lq, B, E, generator=torch.Generator().manual_seed(6)).to(dev)
    (o.float() * g).sum().backward()
    qd, kd, vd = [t.detach().double().clone().requires_grad_(True) for t in (qb, kb, vb)]
    (_ref(qd, kd, vd, H) * g.double()).sum().backward()
    for a, b in [(qb.grad, qd.grad), (kb.grad, kd.grad), (vb.grad, vd.grad)]:
        rel = (a.double() - b).norm().item() / max(b.norm().item(), 1e-6)
        assert rel < 3e-2, rel


def _nrand(seed, *shape):
    return torch.from_numpy(np.random.default_rng(seed).standard_normal(shape).astype(np.float32))


def test_blocks_match_reference_golden(dev):
    import sys

    from conftest import GOLDEN

    sys.path.insert(0, GOLDEN)
    from weights import fill_state

    from svdformer_pointsea_amd import attention as A

    g = golden("attention.npz")
    tol = dict(atol=2e-5, rtol=2e-5)
    sa = fill_state(A.self_attention(256, 512, nhead=8), seed=100).eval().to(dev)
    x, pos = _nrand(101, 2, 256, 64).to(dev), _nrand(102, 64, 2, 512).to(dev)
    with torch.no_grad():
        np.testing.assert_allclose(sa(x, pos).cpu().numpy(), g["sa_y"], **tol)
        np.testing.assert_allclose(sa(x).cpu().numpy(), g["sa_y_nopos"], **tol)
        ca = fill_state(A.cross_attention(512, 512, nhead=8), seed=110).eval().to(dev)
        y = ca(_nrand(111, 2, 512, 64).to(dev), _nrand(112, 2, 512, 32).to(dev))
        np.testing.assert_allclose(y.cpu().numpy(), g["ca_y"], **tol)
        dec = fill_state(A.SDG_Decoder(512, 64, 8), seed=120).eval().to(dev)
        np.testing.assert_allclose(dec(_nrand(121, 2, 512, 48).to(dev)).cpu().numpy(), g["dec_y"], **tol)
        wo = fill_state(A.self_attention_woinp(768, 768, nhead=8), seed=130).eval().to(dev)
        np.testing.assert_allclose(wo(_nrand(131, 2, 768, 40).to(dev)).cpu().numpy(), g["woinp_y"], **tol)
        sv = fill_state(A.self_attention(384, 256, nhead=4), seed=140).eval().to(dev)
        y = sv(_nrand(141, 2, 384, 3).to(dev), _nrand(142, 3, 2, 256).to(dev))
        np.testing.assert_allclose(y.cpu().numpy(), g["sav_y"], **tol)


def test_block_gradients_match_torch_mha(dev):
    """self_attention backward through our core == through torch's MHA."""
    from svdformer_pointsea_amd import attention as A

    torch.manual_seed(0)
    ours = A.self_attention(64, 128, nhead=4).to(dev)
    ref = torch.nn.MultiheadAttention(128, 4).to(dev)
    ref.load_state_dict(ours.multihead_attn.state_dict())
    x = torch.randn(2, 64, 50, device=dev, requires_grad=True)
    y = ours(x)
    y.square().sum().backward()
    g_ours = [p.grad.clone() for p in ours.multihead_attn.parameters()]
    # same block with torch's MHA swapped in
    ours.zero_grad()
    mha = ours.multihead_attn
    ours.multihead_attn = ref
    x2 = x.detach().clone().requires_grad_(True)
    ours(x2).square().sum().backward()
    for a, p in zip(g_ours, ref.parameters()):
        torch.testing.assert_close(a, p.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-4, atol=1e-5)
    ours.multihead_attn = mha
