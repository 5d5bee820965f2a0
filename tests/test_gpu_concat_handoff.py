"""GPU tests of the round-6 glue removals in the SDG refinement stage (SVDFormer.py:72-86):

- the two decoder outputs written straight into the halves of their concatenation (pcops_add_rows,
  attention._AddToBf16Cat) and the concatenation's gradient handed back as channel slices read in place
  (the strided bf16 hand-off into pcops_layernorm_bwd_ex);
- the SDG query's positional add (`with_pos_embed(src1, pos)`, models/model_utils.py:607) handing its
  bf16 gradient to the LayerNorm that produced src1, summed there in autograd's order.

Every comparison is bitwise against the path it replaces (the module-level A/B switches)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _call(name, *args):
    from svdformer_pointsea_amd._lib import lib

    st = getattr(lib(), name)(*args)
    assert st == 0, (name, st)


@pytest.mark.parametrize("rows,C,ld,dts", [(4096, 512, 1024, (0, 1, 1)), (4096, 512, 1024, (1, 1, 1)),
                                           (333, 64, 192, (0, 0, 0)), (1000, 768, 1536, (0, 1, 1)),
                                           (7, 8, 16, (1, 0, 1))])
def test_add_rows_bitwise(dev, rows, C, ld, dts):
    """pcops_add_rows into a row-strided output = pcops_add's values (torch's promoted-dtype add)."""
    from svdformer_pointsea_amd._lib import ptr, stream_of

    T = {0: torch.float32, 1: torch.bfloat16}
    g = torch.Generator().manual_seed(rows + C)
    a = torch.randn(rows, C, generator=g).to(dev, T[dts[0]])
    b = torch.randn(rows, C, generator=g).to(dev, T[dts[1]])
    out = torch.full((rows, ld), 7.0, device=dev, dtype=T[dts[2]])
    off = ld - C
    _call("pcops_add_rows", ptr(a), dts[0], ptr(b), dts[1], ctypes.c_void_p(out.data_ptr() + off * out.element_size()),
          dts[2], rows, C, ld, stream_of(a))
    torch.cuda.synchronize()
    assert torch.equal(out[:, off:], torch.add(a, b).to(T[dts[2]]))   # torch's promoted-dtype add
    assert (out[:, :off] == 7.0).all()


@pytest.mark.parametrize("rows,C,extra", [(2048, 512, "ld"), (4096, 768, "ld"), (1000, 1024, "ld"),
                                          (2048, 512, "gx"), (513, 768, "gx"), (2048, 512, "gx16")])
@pytest.mark.parametrize("colsum", [False, True])
def test_layernorm_bwd_ex_bitwise(dev, rows, C, extra, colsum):
    """pcops_layernorm_bwd_ex against the entry points it generalises: a row-strided bf16 dy = the
    contiguous copy through pcops_layernorm_bwd_bf16g; dy + dy_x (+ dy16) = pcops_layernorm_bwd(_colsum)
    on the pre-summed fp32 gradient (autograd's widening + accumulation)."""
    from svdformer_pointsea_amd import _lib
    from svdformer_pointsea_amd._lib import lib, ptr, stream_of

    g = torch.Generator().manual_seed(rows * 3 + C + colsum)
    a = torch.randn(rows, C, generator=g).to(dev)
    b = torch.randn(rows, C, generator=g).to(dev, torch.bfloat16)
    w = (1 + 0.1 * torch.randn(C, generator=g)).to(dev)
    x = a + b.float()
    mean = x.mean(1)
    rstd = 1.0 / torch.sqrt(x.var(1, unbiased=False) + 1e-5)
    wide = torch.randn(rows, 2 * C, generator=g).to(dev, torch.bfloat16)
    g16 = torch.randn(rows, C, generator=g).to(dev, torch.bfloat16)
    g32 = torch.randn(rows, C, generator=g).to(dev)
    gx = torch.randn(rows, C, generator=g).to(dev, torch.bfloat16)
    sflag = 1 if colsum else 0   # dsum over dx16 (b's dtype), stored fp32

    def outs():
        return (torch.empty(rows, C, device=dev), torch.empty(rows, C, device=dev, dtype=torch.bfloat16),
                torch.empty(C, device=dev), torch.empty(C, device=dev),
                torch.empty(C, device=dev) if colsum else None)

    wsb = (lib().pcops_layernorm_bwd_colsum_workspace_bytes(rows, C) if colsum
           else lib().pcops_layernorm_bwd_workspace_bytes(rows, C))
    ws = _lib.Workspace.get(dev, wsb)
    s = stream_of(a)
    got, ref = outs(), outs()
    common = (ptr(a), 0, ptr(b), 1, ptr(w), ptr(mean), ptr(rstd), rows, C)

    def tail(o):
        return (ptr(o[0]), ptr(o[1]), ptr(o[2]), ptr(o[3]), ptr(o[4]), sflag if colsum else 0, ptr(ws), wsb, s)

    if extra == "ld":
        dy = wide[:, C:]
        _call("pcops_layernorm_bwd_ex", ptr(dy), 1, 2 * C, None, ptr(g16), *common, *tail(got))
        _call("pcops_layernorm_bwd_bf16g", ptr(dy.contiguous()), ptr(g16), *common, *tail(ref))
    else:
        h16 = g16 if extra == "gx16" else None
        _call("pcops_layernorm_bwd_ex", ptr(g32), 0, C, ptr(gx), ptr(h16), *common, *tail(got))
        pre = g32 + gx.float()
        if colsum:
            _call("pcops_layernorm_bwd_colsum", ptr(pre), ptr(h16), *common, *tail(ref))
        else:
            _call("pcops_layernorm_bwd", ptr(pre), ptr(h16), *common, ptr(ref[0]), ptr(ref[1]), ptr(ref[2]),
                  ptr(ref[3]), ptr(ws), wsb, s)
    torch.cuda.synchronize()
    for u, v in zip(got, ref):
        if u is not None:
            assert torch.equal(u, v)


def test_layernorm_bwd_ex_rejects(dev):
    from svdformer_pointsea_amd._lib import lib, ptr, stream_of

    a = torch.zeros(16, 64, device=dev)
    w = torch.ones(64, device=dev)
    d = torch.zeros(16, 64, device=dev, dtype=torch.bfloat16)
    args = (ptr(a), 0, None, 0, ptr(w), ptr(w), ptr(w), 16, 64, ptr(a), None, ptr(w), ptr(w), None, 0, ptr(a), 1 << 20,
            stream_of(a))
    assert lib().pcops_layernorm_bwd_ex(ptr(d), 1, 60, None, None, *args) != 0        # ld < C
    assert lib().pcops_layernorm_bwd_ex(ptr(d), 1, 68, None, None, *args) != 0        # ld % 8
    assert lib().pcops_layernorm_bwd_ex(ptr(d), 1, 64, ptr(d), None, *args) != 0      # dy_x with bf16 dy
    assert lib().pcops_add_rows(ptr(a), 0, ptr(a), 0, ptr(a), 0, 16, 64, 32, stream_of(a)) != 0   # ld < C


@pytest.mark.parametrize("L,C1,C2", [(512, 256, 256), (2048, 512, 512), (300, 256, 512)])
def test_block_sum_cat_bitwise(dev, monkeypatch, L, C1, C2):
    """block_sum_cat (both sums written into the concatenation, its gradient read as channel slices)
    against block_sum + torch.cat: the concatenation and every input / parameter gradient bitwise,
    through a conv_ps-like Linear that reads the concatenation."""
    import svdformer_pointsea_amd.attention as A

    torch.manual_seed(L + C1 + C2)
    b1 = A.self_attention(C1, C1, nhead=8).to(dev)
    b2 = A.self_attention(C1, C2, nhead=8).to(dev)
    ps = torch.nn.Linear(C1 + C2, 2 * C2).to(dev)
    x0 = torch.randn(2, L, C1, device=dev)
    g = torch.randn(2, L, 2 * C2, device=dev)
    mods = (b1, b2, ps)

    def run(on):
        monkeypatch.setattr(A, "_CAT_ROWS", on)
        for m in mods:
            m.zero_grad()
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            t = A.block_sum_cat(b1.forward_tokens(x), b2.forward_tokens(x))
            y = A.linear(t, ps.weight, ps.bias)
        y.float().backward(g)
        return [t.detach(), x.grad] + [p.grad.clone() for m in mods for p in m.parameters()]

    got, ref = run(True), run(False)
    assert got[0].dtype == torch.bfloat16 and got[0].shape == (2, L, C1 + C2)
    for u, v in zip(got, ref):
        assert torch.equal(u, v)


@pytest.mark.parametrize("kind", ["self", "cross"])
@pytest.mark.parametrize("L,C", [(512, 256), (2048, 512), (300, 768)])
def test_pos_grad_mailbox_bitwise(dev, monkeypatch, kind, L, C):
    """The SDG query's positional add handing its bf16 gradient to the LayerNorm that produced the query
    (summed inside pcops_layernorm_bwd_ex after the residual's fp32 gradient) against the widening cast +
    autograd accumulation: input and parameter gradients bitwise.  self: the LayerNorm's bf16 copy also
    feeds v (dy16 present); cross: it feeds nothing else (dy16 absent)."""
    import svdformer_pointsea_amd.attention as A
    from svdformer_pointsea_amd.svdformer import SinusoidalPositionalEmbedding

    torch.manual_seed(L + C)
    blk = (A.self_attention(C, C, nhead=8) if kind == "self" else A.cross_attention(C, C, nhead=8)).to(dev)
    emb = SinusoidalPositionalEmbedding(C).to(dev)
    x0 = torch.randn(2, L, C, device=dev)
    k0 = torch.randn(2, L // 2 + 3, C, device=dev)
    cd = torch.rand(2, L, device=dev) * 20
    g = torch.randn(2, L, C, device=dev).to(torch.bfloat16)

    def run(on):
        monkeypatch.setattr(A, "_POS_GX", on)
        blk.zero_grad()
        x = x0.clone().requires_grad_(True)
        k = k0.clone().requires_grad_(True)
        pos = A.PosEmbedding(cd, emb, C)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            s, f = blk.forward_tokens(x, pos) if kind == "self" else blk.forward_tokens(x, k, pos)
            y = A.block_sum(s, f, True)
        y.backward(g)
        out = [x.grad] + [p.grad.clone() for p in blk.parameters() if p.grad is not None]
        if kind == "cross":
            out.append(k.grad)
        return out

    got, ref = run(True), run(False)
    assert len(got) == len(ref)
    for u, v in zip(got, ref):
        assert torch.equal(u, v)


@pytest.mark.parametrize("dataset", ["PCN", "ShapeNet"])
def test_sdg_refine_glue_bitwise(dev, monkeypatch, dataset):
    """The refinement stage (SDG, SVDFormer.py:38-104) with both changes on against both off: output and
    every gradient bitwise -- with self_attention decoders ("PCN") and with SDG_Decoder (the bench
    model's PCNConfig, TEST_DATASET "ShapeNet": its sa2 pair reaches the concatenation)."""
    import svdformer_pointsea_amd.attention as A
    from svdformer_pointsea_amd.svdformer import SDG

    torch.manual_seed(5)
    sdg = SDG(ratio=2, hidden_dim=512, dataset=dataset).to(dev)
    B, N = 2, 256
    local0 = torch.randn(B, 512, 256, device=dev) * 0.1
    coarse0 = torch.rand(B, N, 3, device=dev)
    fg0 = torch.randn(B, 512, 1, device=dev)
    part0 = torch.rand(B, 2048, 3, device=dev)

    def run(on):
        monkeypatch.setattr(A, "_CAT_ROWS", on)
        monkeypatch.setattr(A, "_POS_GX", on)
        sdg.zero_grad()
        local, coarse, fg = (t.clone().requires_grad_(True) for t in (local0, coarse0, fg0))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = sdg.forward_tokens(local, coarse, fg, part0)
        out.float().square().sum().backward()
        return [out.detach(), local.grad, coarse.grad, fg.grad] + [
            p.grad.clone() for p in sdg.parameters() if p.grad is not None]

    got, ref = run(True), run(False)
    assert len(got) == len(ref)
    for u, v in zip(got, ref):
        assert torch.equal(u, v)
