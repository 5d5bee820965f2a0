"""The data-parallel gradient path on the GPU with a real RCCL process group
(one rank: the one-GPU box's stand-in for the 8-GPU node): the bucketed
all-reduce issued from backward hooks (train.BucketedAllReduce) -- eagerly
and captured inside a HIP graph -- must give the gradients of the single
all-reduce after backward, bitwise, on the bf16-shadow + fp32 parameter
layout bench.py uses."""
import copy
import socket
import time

import pytest
import torch
import torch.distributed as dist
from torch import nn

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def group(dev):
    owned = not dist.is_initialized()
    if owned:
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                device_id=dev)
    yield
    if owned:
        torch.cuda.synchronize()
        dist.destroy_process_group()


class _Net(nn.Module):
    def __init__(self):
        super().__init__()
        from svdformer_pointsea_amd.attention import self_attention

        self.blk = self_attention(32, 64, nhead=2)
        self.norm = nn.LayerNorm(64)
        self.head = nn.Linear(64, 3)
        self.side = nn.Linear(32, 48)
        self.unused = nn.Linear(5, 5)
        # fp32 (LayerNorm) parameters after the head: with tiny buckets they form
        # several fp32 buckets gathered on the communication stream while the
        # rest of backward still allocates on the compute stream
        self.post = nn.ModuleList(nn.LayerNorm(3) for _ in range(3))

    def forward(self, x):
        from svdformer_pointsea_amd import _lib

        # a branch on a side stream (as the model's local encoder): its weight
        # gradients are produced on that stream during backward
        with _lib.fork(x.device, lane=3, inputs=(x,)) as br:
            z = self.side(x.mean(2))
        y = self.blk(x).transpose(1, 2)
        h = self.head(self.norm(y.float())).float()
        for m in self.post:
            h = m(h) * 1.5 + h
        return h.square().mean() + br.join(z).float().square().mean()


def _step(fp, x, sync):
    fp.zero_grad()
    fp.refresh()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = fp.forward(x)
    loss.backward()
    if sync is None:
        fp.collect()
        fp.allreduce(1)
    else:
        sync.finish()
    return loss.detach()


@pytest.mark.parametrize("graph,bucket_mb", [(False, 0.01), (True, 0.01), (False, 1e-5), (True, 1e-5)])
def test_bucketed_allreduce_rccl(dev, group, graph, bucket_mb):
    from svdformer_pointsea_amd.train import BucketedAllReduce, FlatParams

    torch.manual_seed(0)
    a = _Net().to(dev)
    b = copy.deepcopy(a)
    x = torch.randn(4, 32, 50, device=dev)
    fa, fb = FlatParams(a, dev), FlatParams(b, dev)
    _step(fa, x, None)
    ref = fa.grad.clone()
    sync = BucketedAllReduce(fb, 1, bucket_mb=bucket_mb)
    assert len(sync.buckets) > 4
    if bucket_mb < 1e-4:   # every parameter its own bucket: several fp32 buckets
        assert sum(1 for _, _, es in sync.buckets if not es[0][3]) >= 4
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            _step(fb, x, sync)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    assert torch.equal(fb.grad, ref)
    if graph:
        # as bench.py captures its collectives: RCCL's watchdog thread polls the eager
        # collectives' events, and under "global" capture such a call from another thread
        # invalidates the capture (the watchdog then aborts the process) -- so drain, let it
        # finish polling, and capture in thread-local mode
        time.sleep(1.0)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            _step(fb, x, sync)
        fb.grad.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(fb.grad, ref), (fb.grad - ref).abs().max().item()
