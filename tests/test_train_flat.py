"""train.FlatParams: bf16 shadows + flat fp32 master/gradient buffers give
exactly the gradients of plain torch.autocast (CPU autocast, bf16)."""
import copy

import torch
from torch import nn

from svdformer_pointsea_amd.train import FlatParams


class _Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv1d(8, 16, 1)
        self.norm = nn.LayerNorm(16)
        self.lin = nn.Linear(16, 4)

    def forward(self, x):
        y = self.conv(x).transpose(1, 2)
        return self.lin(self.norm(y.float())).float().square().mean()


def test_flat_params_match_autocast_grads():
    torch.manual_seed(0)
    a = _Net()
    b = copy.deepcopy(a)
    x = torch.randn(3, 8, 5)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        a(x).backward()
    fp = FlatParams(b, "cpu")
    fp.zero_grad()
    fp.refresh()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        fp.forward(x).backward()
    fp.collect()
    assert fp.n16 == sum(p.numel() for n, p in b.named_parameters() if not n.startswith("norm"))
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert pb.grad.dtype == torch.float32
        assert torch.equal(pa.grad, pb.grad), n
        assert torch.equal(pa.data, pb.data), n
    # the fp32 master weights are the parameters themselves (views of one buffer)
    assert all(p.data_ptr() >= fp.flat.data_ptr() for p in b.parameters())


def test_flat_master_optimizer_equals_per_tensor():
    """Adam / AdamW over FlatParams.master() (one tensor) == per-tensor updates."""
    for make in (lambda ps: torch.optim.Adam(ps, lr=1e-2, betas=(0.9, 0.999)),
                 lambda ps: torch.optim.AdamW(ps, lr=1e-2, weight_decay=5e-4)):
        torch.manual_seed(1)
        a = _Net()
        b = copy.deepcopy(a)
        fa, fb = FlatParams(a, "cpu", bf16=False), FlatParams(b, "cpu", bf16=False)
        oa, ob = make(list(a.parameters())), make([fb.master()])
        for step in range(3):
            x = torch.randn(3, 8, 5, generator=torch.Generator().manual_seed(step))
            for f in (fa, fb):
                f.zero_grad()
                f.forward(x).backward()
            oa.step()
            ob.step()
        assert torch.equal(fa.flat, fb.flat)
        for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
            assert torch.equal(pa.data, pb.data), n


class _Net2(nn.Module):
    """A Linear used twice, a Linear never used, a channels_last Conv2d."""

    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(4, 6, 1).to(memory_format=torch.channels_last)
        self.lin = nn.Linear(6, 6)
        self.unused = nn.Linear(3, 3)

    def forward(self, x):
        y = self.conv(x.contiguous(memory_format=torch.channels_last)).flatten(2).transpose(1, 2)
        return self.lin(torch.relu(self.lin(y))).float().square().mean()


def test_flat_params_reused_unused_and_channels_last():
    torch.manual_seed(3)
    a = _Net2()
    b = copy.deepcopy(a)
    x = torch.randn(2, 4, 3, 5)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        a(x).backward()
    fp = FlatParams(b, "cpu")
    assert b.conv.weight.is_contiguous(memory_format=torch.channels_last)
    for _ in range(2):   # the second step must not accumulate into the first
        fp.zero_grad()
        fp.refresh()
        with torch.autocast("cpu", dtype=torch.bfloat16):
            fp.forward(x).backward()
        fp.collect()
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        ref = torch.zeros_like(pa) if pa.grad is None else pa.grad
        assert torch.equal(ref, pb.grad), n


class _Net3(nn.Module):
    """A Conv2d block built with if_bn=False (its BatchNorm is never read, as
    models/model_utils.py:27-43) beside a used LayerNorm."""

    def __init__(self):
        super().__init__()
        from svdformer_pointsea_amd.svdformer import Conv2d

        self.block = Conv2d(4, 6, if_bn=False)
        self.norm = nn.LayerNorm(6)
        with torch.no_grad():
            self.block.bn.weight.fill_(1.5)
            self.block.bn.bias.fill_(0.25)

    def forward(self, x):
        return self.norm(self.block(x).flatten(2).transpose(1, 2)).square().mean()


def test_flat_adamw_leaves_never_used_parameters_alone():
    """AdamW (weight decay 5e-4, the PointSea loop) over FlatParams.master()
    == per-tensor AdamW, which skips parameters whose .grad is None: the
    if_bn=False BatchNorm keeps its values instead of being decayed."""
    from svdformer_pointsea_amd.train import never_used

    torch.manual_seed(4)
    a = _Net3()
    b = copy.deepcopy(a)
    assert never_used(b) == {"block.bn.weight", "block.bn.bias"}
    oa = torch.optim.AdamW(a.parameters(), lr=1e-2, weight_decay=5e-4)
    fb = FlatParams(b, "cpu", bf16=False)
    ob = torch.optim.AdamW([fb.master()], lr=1e-2, weight_decay=5e-4)
    for step in range(3):
        x = torch.randn(2, 4, 3, 5, generator=torch.Generator().manual_seed(step))
        oa.zero_grad(set_to_none=True)
        a(x).backward()
        oa.step()
        fb.zero_grad()
        fb.forward(x).backward()
        ob.step()
    assert a.block.bn.weight.grad is None
    assert torch.equal(b.block.bn.weight, torch.full((6,), 1.5)) and torch.equal(b.block.bn.bias, torch.full((6,), 0.25))
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(pa.data, pb.data), n


def test_lr_schedule_matches_reference_scheduler():
    """train.TrainSchedule (warm-up per batch for 300 batches, then MultiStepLR /
    StepLR per epoch) == the reference's GradualWarmupScheduler driven by its
    loops (tests/golden/make_golden_train.py), also with a tensor LR (what a
    graph-captured fused Adam reads)."""
    import warnings

    import numpy as np

    from conftest import golden
    from svdformer_pointsea_amd.train import TrainSchedule

    g = golden("lr_schedule.npz")
    for policy, model in (("pcn", "svdformer"), ("55", "pointsea")):
        for lr0 in (1e-4, torch.tensor(1e-4, dtype=torch.float64)):
            p = torch.nn.Parameter(torch.zeros(1))
            opt = torch.optim.Adam([p], lr=lr0)
            sch = TrainSchedule(opt, model)
            lrs = []
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                for _ in range(90):
                    for _ in range(7):
                        lrs.append(float(opt.param_groups[0]["lr"]))
                        sch.batch_end()
                    sch.epoch_end()
            np.testing.assert_allclose(np.array(lrs), g[policy], rtol=1e-12, atol=0)


def test_checkpoint_interop_with_per_tensor_optimizer():
    """checkpoint_state(FlatParams) == the reference's checkpoint of a
    per-tensor Adam (core/train_pcn.py:152-166: 'module.'-prefixed model keys,
    per-parameter optimizer state); loading it back (into the flat optimizer,
    or a reference-style checkpoint into it) continues identically."""
    from svdformer_pointsea_amd.train import checkpoint_state, load_checkpoint_state

    torch.manual_seed(5)
    a = _Net3()
    b = copy.deepcopy(a)
    oa = torch.optim.Adam(a.parameters(), lr=1e-2)
    fb = FlatParams(b, "cpu", bf16=False)
    ob = torch.optim.Adam([fb.master()], lr=1e-2)

    def train(step_fn, steps, seed0):
        for step in range(steps):
            step_fn(torch.randn(2, 4, 3, 5, generator=torch.Generator().manual_seed(seed0 + step)))

    def sa(x):
        oa.zero_grad(set_to_none=True)
        a(x).backward()
        oa.step()

    def sb(x, fb=fb, ob=ob):
        fb.zero_grad()
        fb.forward(x).backward()
        ob.step()

    train(sa, 2, 0)
    train(sb, 2, 0)
    ref = {"model": {"module." + k: v for k, v in a.state_dict().items()}, "optimizer": oa.state_dict()}
    got = checkpoint_state(b, ob, fb)
    assert got["model"].keys() == ref["model"].keys()
    assert all(torch.equal(got["model"][k], ref["model"][k]) for k in ref["model"])
    assert got["optimizer"]["state"].keys() == ref["optimizer"]["state"].keys()
    for i, ent in ref["optimizer"]["state"].items():
        for k, v in ent.items():
            assert torch.equal(got["optimizer"]["state"][i][k], v), (i, k)
    # a reference-style checkpoint loaded into a fresh flat model + optimizer
    c = _Net3()
    fc = FlatParams(c, "cpu", bf16=False)
    oc = torch.optim.Adam([fc.master()], lr=1e-2)
    load_checkpoint_state(ref, c, oc, fc)
    train(sa, 2, 10)
    train(lambda x: sb(x, fc, oc), 2, 10)
    for (n, pa), (_, pc) in zip(a.named_parameters(), c.named_parameters()):
        assert torch.equal(pa.data, pc.data), n


def test_checkpoint_from_capturable_tensor_lr_optimizer_loads_into_plain_adam():
    """bench.py's optimizer is capturable with a tensor LR (a captured graph reads it);
    its checkpoint must still be the reference's: host-float lr, default fused /
    capturable / foreach, host step -- a plain per-tensor Adam loads it and then
    steps exactly like the optimizer that wrote it."""
    from svdformer_pointsea_amd.train import checkpoint_state

    torch.manual_seed(6)
    a = _Net3()
    b = copy.deepcopy(a)
    fb = FlatParams(b, "cpu", bf16=False)
    ob = torch.optim.Adam([fb.master()], lr=torch.tensor(1e-2), foreach=False)
    oa = torch.optim.Adam(a.parameters(), lr=1e-2)
    for step in range(2):
        x = torch.randn(2, 4, 3, 5, generator=torch.Generator().manual_seed(step))
        fb.zero_grad()
        fb.forward(x).backward()
        ob.step()
        oa.zero_grad(set_to_none=True)
        a(x).backward()
        oa.step()
    # the group flags bench.py's CUDA optimizer carries (capturable / fused need a GPU here)
    ob.param_groups[0].update(capturable=True, fused=True)
    ck = checkpoint_state(b, ob, fb)
    (g,) = ck["optimizer"]["param_groups"]
    assert isinstance(g["lr"], float) and g["capturable"] is False and g["fused"] is None and g["foreach"] is None
    assert all(not ent["step"].is_cuda and ent["step"].dtype == torch.float32 for ent in ck["optimizer"]["state"].values())
    c = _Net3()
    c.load_state_dict({k[len("module."):]: v for k, v in ck["model"].items()})
    oc = torch.optim.Adam(c.parameters(), lr=1e-2)
    oc.load_state_dict(ck["optimizer"])
    assert oc.param_groups[0]["capturable"] is False
    x = torch.randn(2, 4, 3, 5, generator=torch.Generator().manual_seed(9))
    for opt, m in ((oa, a), (oc, c)):
        opt.zero_grad(set_to_none=True)
        m(x).backward()
        opt.step()
    for (n, pa), (_, pc) in zip(a.named_parameters(), c.named_parameters()):
        torch.testing.assert_close(pc.data, pa.data, rtol=1e-6, atol=1e-7, msg=n)


def test_checkpoint_roundtrip_keeps_tensor_lr_and_switches():
    """reloading this repo's own checkpoint (reference layout: float lr,
    default switches) into bench.py's kind of flat optimizer (tensor LR a captured
    graph reads, explicit implementation switches) keeps that LR tensor object --
    the saved value written into it -- and the live switches, and then steps
    exactly like the optimizer that wrote the checkpoint."""
    from svdformer_pointsea_amd.train import checkpoint_state, load_checkpoint_state

    torch.manual_seed(7)
    a = _Net3()
    b = copy.deepcopy(a)
    fa = FlatParams(a, "cpu", bf16=False)
    oa = torch.optim.Adam([fa.master()], lr=torch.tensor(1e-2), foreach=False)
    for step in range(2):
        x = torch.randn(2, 4, 3, 5, generator=torch.Generator().manual_seed(step))
        fa.zero_grad()
        fa.forward(x).backward()
        oa.step()
    ck = checkpoint_state(a, oa, fa)
    fb = FlatParams(b, "cpu", bf16=False)
    lr_t = torch.tensor(0.5)
    ob = torch.optim.Adam([fb.master()], lr=lr_t, foreach=False)
    load_checkpoint_state(ck, b, ob, fb)
    g = ob.param_groups[0]
    assert g["lr"] is lr_t and float(lr_t) == float(torch.tensor(1e-2))
    assert g["foreach"] is False
    x = torch.randn(2, 4, 3, 5, generator=torch.Generator().manual_seed(9))
    for f, o in ((fa, oa), (fb, ob)):
        f.zero_grad()
        f.forward(x).backward()
        o.step()
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(pa.data, pb.data), n


import pytest  # noqa: E402


@pytest.mark.gpu
def test_checkpoint_roundtrip_capturable_flat_optimizer_gpu():
    """The same round trip into a capturable, tensor-LR flat Adam on the GPU
    (bench.py's optimizer): capturable stays on, the step stays on the device,
    the captured LR tensor is kept, and the next step equals the writer's."""
    from svdformer_pointsea_amd.train import checkpoint_state, load_checkpoint_state

    dev = "cuda"
    torch.manual_seed(8)
    a = _Net3().to(dev)
    b = copy.deepcopy(a)
    fa = FlatParams(a, dev, bf16=False)
    oa = torch.optim.Adam([fa.master()], lr=torch.tensor(1e-2, device=dev), capturable=True, foreach=False)
    for step in range(2):
        x = torch.randn(2, 4, 3, 5, generator=torch.Generator().manual_seed(step)).to(dev)
        fa.zero_grad()
        fa.forward(x).backward()
        oa.step()
    ck = checkpoint_state(a, oa, fa)
    fb = FlatParams(b, dev, bf16=False)
    lr_t = torch.tensor(0.5, device=dev)
    ob = torch.optim.Adam([fb.master()], lr=lr_t, capturable=True, foreach=False)
    load_checkpoint_state(ck, b, ob, fb)
    g = ob.param_groups[0]
    assert g["capturable"] is True and g["lr"] is lr_t
    (st,) = ob.state.values()
    assert st["step"].is_cuda
    x = torch.randn(2, 4, 3, 5, generator=torch.Generator().manual_seed(9)).to(dev)
    for f, o in ((fa, oa), (fb, ob)):
        f.zero_grad()
        f.forward(x).backward()
        o.step()
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(pa.data, pb.data), n


class _NetMix(nn.Module):
    """Linear layers (bf16 shadows) around a LayerNorm (fp32 region), sizes not multiples of 4."""

    def __init__(self):
        super().__init__()
        self.l1 = nn.Linear(37, 129)
        self.norm = nn.LayerNorm(129)
        self.l2 = nn.Linear(129, 19)

    def forward(self, x):
        return self.l2(self.norm(self.l1(x)).relu()).square().mean()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,bf16_grads", [("adam", True), ("adamw", True), ("adam", False)])
def test_flat_adam_matches_torch_fused(kind, bf16_grads):
    """train.FlatAdam (pcops_adam_flat: bf16 shadow-region gradients read from the bf16 bucket, the new
    shadows written by the update; bf16_grads=False: the whole fp32 bucket, the data-parallel path's)
    against torch's fused capturable Adam / AdamW on the same flat
    buffers: master weights and both moments within fp32 rounding of torch's (the kernel's
    arithmetic order is torch's; torch forms some products in double), shadows = bf16(master), the
    torch optimizer's state_dict layout unchanged."""
    from svdformer_pointsea_amd.train import FlatAdam

    dev = "cuda"
    torch.manual_seed(4)
    a = _NetMix().to(dev)
    b = copy.deepcopy(a)
    fa, fb = FlatParams(a, dev), FlatParams(b, dev)
    mk = (lambda ps, lr: torch.optim.Adam(ps, lr=lr, betas=(0.9, 0.999), weight_decay=0, fused=True,
                                          capturable=True)) if kind == "adam" else \
         (lambda ps, lr: torch.optim.AdamW(ps, lr=lr, weight_decay=5e-4, fused=True, capturable=True))
    oa = mk([fa.master()], torch.tensor(1e-3, device=dev))
    ob = mk([fb.master()], torch.tensor(1e-3, device=dev))
    flat = FlatAdam(ob, fb)
    fb.refresh()
    for step in range(5):
        x = torch.randn(64, 37, generator=torch.Generator().manual_seed(step)).to(dev)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            fa.zero_grad()
            fa.refresh()
            fa.forward(x).backward()
            fb.zero_grad()
            fb.forward(x).backward()
        fa.collect()
        fb.collect(widen=not bf16_grads)
        oa.step()
        flat.step(bf16_grads=bf16_grads)
        torch.testing.assert_close(fb.flat, fa.flat, rtol=2e-6, atol=1e-8)
    (sa,), (sb,) = oa.state.values(), ob.state.values()
    assert sorted(sa) == sorted(sb) and torch.equal(sa["step"], sb["step"])
    torch.testing.assert_close(sb["exp_avg"], sa["exp_avg"], rtol=2e-6, atol=1e-10)
    torch.testing.assert_close(sb["exp_avg_sq"], sa["exp_avg_sq"], rtol=2e-6, atol=1e-14)
    assert torch.equal(fb.flat16, fb.flat[:fb.n16].to(torch.bfloat16))


@pytest.mark.gpu
def test_flat_adam_validates_state_and_lr():
    """FlatAdam hands the kernel raw pointers to the step counter and a tensor LR: a step
    kept as a Python number or a host / float64 tensor (a non-capturable optimizer, an old checkpoint)
    is converted to a device fp32 tensor before use; a tensor LR that is not a 0-dim fp32 tensor on the
    master's device is refused; Adam(decoupled_weight_decay=True) takes the AdamW update."""
    from svdformer_pointsea_amd.train import FlatAdam

    dev = "cuda"
    torch.manual_seed(5)
    fp = FlatParams(_NetMix().to(dev), dev)
    with pytest.raises(ValueError, match="tensor lr"):
        FlatAdam(torch.optim.Adam([fp.master()], lr=torch.tensor(1e-3), fused=True), fp)        # host LR
    with pytest.raises(ValueError, match="tensor lr"):
        FlatAdam(torch.optim.Adam([fp.master()], lr=torch.tensor(1e-3, dtype=torch.float64, device=dev),
                                  capturable=True), fp)
    opt = torch.optim.Adam([fp.master()], lr=1e-3, decoupled_weight_decay=True, weight_decay=1e-2)
    flat = FlatAdam(opt, fp)
    assert flat.adamw
    p = opt.param_groups[0]["params"][0]   # the optimizer's own key (master() returns a new view)
    for step in (3, torch.tensor(3.0), torch.tensor(3.0, dtype=torch.float64)):
        opt.state[p] = {"step": step, "exp_avg": torch.zeros_like(p), "exp_avg_sq": torch.zeros_like(p)}
        x = torch.randn(8, 37, device=dev)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            fp.zero_grad()
            fp.refresh()
            fp.forward(x).backward()
        fp.collect()
        flat.step(bf16_grads=False)
        st = opt.state[p]["step"]
        assert st.is_cuda and st.dtype == torch.float32 and float(st) == 4.0


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["svdformer", "pointsea"])
def test_captured_flat_adam_follows_lr_schedule(model):
    """bench.py's optimizer path (VERDICT r4 hygiene): FlatAdam over a fused capturable Adam (PCN) /
    AdamW (ShapeNet-55) whose LR is a device tensor, the update captured ONCE into a HIP graph and
    replayed, TrainSchedule.batch_end() between replays (epoch_end every 7 batches, as the golden's
    loop).  Before replay i the LR tensor the graph reads holds golden[i] (the reference's
    GradualWarmupScheduler sequence, tests/golden/make_golden_train.py) to fp32 rounding -- the
    schedule does its arithmetic on the fp32 device tensor -- and after it the master weights equal,
    bitwise, an eager FlatAdam handed that same value as a host number: the graph applies the live
    LR, not the one at capture.  No scheduler warning is raised (FlatAdam flags its step as the
    optimizer's)."""
    import warnings

    import numpy as np

    from conftest import golden
    from svdformer_pointsea_amd.train import FlatAdam, TrainSchedule

    dev = "cuda"
    gold = golden("lr_schedule.npz")["pcn" if model == "svdformer" else "55"]
    torch.manual_seed(11)
    a = _NetMix().to(dev)
    b = copy.deepcopy(a)
    fa, fb = FlatParams(a, dev), FlatParams(b, dev)
    mk = (lambda ps, lr: torch.optim.Adam(ps, lr=lr, betas=(0.9, 0.999), weight_decay=0, fused=True,
                                          capturable=True)) if model == "svdformer" else \
         (lambda ps, lr: torch.optim.AdamW(ps, lr=lr, weight_decay=0.0005, fused=True, capturable=True))
    lr_t = torch.tensor(1e-4, device=dev)
    oa, ob = mk([fa.master()], lr_t), mk([fb.master()], 1e-4)
    fla, flb = FlatAdam(oa, fa), FlatAdam(ob, fb)
    fa.refresh()
    fb.refresh()
    gen = torch.Generator(device=dev).manual_seed(3)
    for f in (fa, fb):   # one fixed gradient (bf16 shadow region + fp32 region), the same on both
        f.grad16.copy_(torch.randn(f.grad16.shape, generator=gen.manual_seed(3), device=dev))
        f.grad.copy_(torch.randn(f.grad.shape, generator=gen.manual_seed(4), device=dev))
    graph = None
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        sch = TrainSchedule(oa, model)
        for i, want in enumerate(gold):
            lr_now = float(oa.param_groups[0]["lr"])
            assert oa.param_groups[0]["lr"] is lr_t
            # fp32 rounding, compounded over StepLR's per-epoch x0.98 (measured worst 8e-7 on the CPU)
            np.testing.assert_allclose(lr_now, want, rtol=2e-6, atol=0, err_msg=f"batch {i}")
            if graph is None:     # the first update eagerly (creates the state), then captured once
                fla.step()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    fla.step()
            else:
                graph.replay()
            ob.param_groups[0]["lr"] = lr_now
            flb.step()
            sch.batch_end()
            if (i + 1) % 7 == 0:
                sch.epoch_end()
            assert torch.equal(fa.flat, fb.flat), f"batch {i}: master differs (lr {lr_now})"
    assert torch.equal(fa.flat16, fb.flat16)
    bad = [str(w.message) for w in caught if "lr_scheduler" in str(w.message) or "optimizer.step" in str(w.message)]
    assert not bad, bad
