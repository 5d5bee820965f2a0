"""pcops_linear_skinny (EdgeConv's first-layer 1x1 convs, models/model_utils.py:847-881) against the fp32
expression it computes and against torch's bf16 GEMM, and the EdgeConv module with it on against off."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _skinny(x, A, b, N):
    from svdformer_pointsea_amd._lib import lib, ptr, stream_of

    y = torch.full((x.shape[0], N), float("nan"), dtype=torch.bfloat16, device=x.device)
    st = lib().pcops_linear_skinny(ptr(x), x.shape[0], x.shape[1], ptr(A), ptr(b), ptr(y), N, stream_of(x))
    assert st == 0, st
    torch.cuda.synchronize()
    return y


def _ulp_close(got, ref, mag, exact_frac=0.995):
    """got (bf16) within one bf16 spacing of ref (float64 or bf16) plus the fp32 accumulation bound
    (K ulps of fp32 of the terms' magnitude `mag` = sum |x_k A_nk| + |b_n|: an output that cancels to
    far below its terms carries that absolute error, many of ITS bf16 spacings), and equal to ref's
    bf16 rounding on almost every element."""
    r = ref.double()
    d = (got.double() - r).abs()
    spacing = torch.exp2(torch.floor(torch.log2(r.abs().clamp_min(2.0 ** -126))) - 7)
    bound = spacing + mag * 2.0 ** -18
    assert torch.isfinite(got.float()).all()
    assert (d <= bound).all(), float((d / bound).max())
    assert (got == ref.to(torch.bfloat16)).float().mean().item() > exact_frac


@pytest.mark.parametrize("rows", [1, 31, 33, 1000, 1 << 20])
@pytest.mark.parametrize("K,N", [(6, 32), (32, 32), (32, 64), (64, 32), (6, 64), (64, 64)])
@pytest.mark.parametrize("bias", [True, False])
def test_linear_skinny_matches_fp32(dev, rows, K, N, bias):
    if rows == 1 << 20 and (K, N) not in ((6, 32), (32, 64)):
        pytest.skip("the full edge-row count at the gcn_1 shapes only")
    g = torch.Generator().manual_seed(rows + K * 7 + N)
    x = torch.randn(rows, K, generator=g).to(dev, torch.bfloat16)
    A = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev, torch.bfloat16)
    b = torch.randn(N, generator=g).to(dev, torch.bfloat16) if bias else None
    y = _skinny(x, A, b, N)
    ref = x.double() @ A.double().t()   # products of bf16 values and their sum, exact to float64
    mag = x.double().abs() @ A.double().abs().t()
    if bias:
        ref = ref + b.double()
        mag = mag + b.double().abs()
    _ulp_close(y, ref, mag)
    # torch's bf16 GEMM (the path it replaces): the same values up to the accumulation order
    tb = torch.nn.functional.linear(x, A, b)
    _ulp_close(y, tb, 2 * mag, exact_frac=0.99)
    # deterministic
    assert torch.equal(y, _skinny(x, A, b, N))


def test_linear_skinny_rejects(dev):
    from svdformer_pointsea_amd._lib import lib, ptr, stream_of

    x = torch.zeros(64, 32, dtype=torch.bfloat16, device=dev)
    A = torch.zeros(48, 32, dtype=torch.bfloat16, device=dev)
    y = torch.zeros(64, 48, dtype=torch.bfloat16, device=dev)
    assert lib().pcops_linear_skinny(ptr(x), 64, 32, ptr(A), None, ptr(y), 48, stream_of(x)) != 0   # N % 32
    assert lib().pcops_linear_skinny(ptr(x), 64, 16, ptr(A), None, ptr(y), 32, stream_of(x)) != 0   # K
    odd = ctypes.c_void_p(x.data_ptr() + 8)
    assert lib().pcops_linear_skinny(odd, 32, 32, ptr(A), None, ptr(y), 32, stream_of(x)) != 0      # alignment


def test_linear_skinny_unaligned_weight(dev):
    """A (the conv weight) may sit at any bf16 offset of the flat parameter buffer."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4096, 6, generator=g).to(dev, torch.bfloat16)
    flat = torch.randn(1 + 32 * 6 + 32, generator=g).to(dev, torch.bfloat16)
    A, b = flat[1:1 + 192].view(32, 6), flat[193:]
    y = _skinny(x, A, b, 32)
    assert torch.equal(y, _skinny(x, A.contiguous().clone(), b.clone(), 32))


@pytest.mark.parametrize("cin,cout,k,N", [(3, 64, 16, 2048), (3, 64, 16, 300)])
def test_edgeconv_skinny_on_off(dev, monkeypatch, cin, cout, k, N):
    """EdgeConv (gcn_1's shape) with the skinny convs against the GEMM library's: outputs and every
    gradient within bf16 tolerance (the two differ only in the fp32 accumulation order inside each
    conv); the skinny path's output and parameter gradients bitwise run to run."""
    import svdformer_pointsea_amd.attention as A
    from svdformer_pointsea_amd.svdformer import EdgeConv

    torch.manual_seed(cin + cout + N)
    m = EdgeConv(cin, cout, k).to(dev)
    x0 = torch.rand(4, cin, N, device=dev)
    g = torch.randn(4, cout, N, device=dev)

    def run(on):
        monkeypatch.setattr(A, "_SKINNY", on)   # off by default (no step gain); tested both ways
        m.zero_grad()
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        y.float().backward(g)
        return [y.detach().float(), x.grad] + [p.grad.clone() for p in m.parameters()]

    on, on2, off = run(True), run(True), run(False)
    for i, (a, b) in enumerate(zip(on, on2)):
        if i == 1:   # the input gradient: edge_group_grad scatters by fp32 atomics (order-dependent)
            assert float((a - b).abs().max()) <= 1e-5 * (float(a.abs().max()) + 1e-6)
        else:
            assert torch.equal(a, b)
    for a, b in zip(on, off):
        scale = float(b.abs().max()) + 1e-6
        assert float((a - b).abs().max()) <= 2e-2 * scale, (float((a - b).abs().max()), scale)
