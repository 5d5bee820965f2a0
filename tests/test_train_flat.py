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
