"""BatchNorm (+ReLU) forward and backward times at the ResNet shapes of the PCN step (96 depth
images, channels_last bf16), fused final on and off (PCOPS_BN_FUSED_FINAL is read per call):
10 forward + backward calls captured in a HIP graph, HIP events around its replays (no host
time in the figure).  PCOPS_LIB_PATH selects an A/B build.
    python tools/bn_bench.py"""
import os
import sys

import torch
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svdformer_pointsea_amd.batchnorm import ACT_RELU, bn_act  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = [(96, 16, 224, 224), (96, 32, 112, 112), (96, 64, 56, 56), (96, 128, 28, 28)]
tag = os.environ.get("PCOPS_LIB_PATH", "default")


def graph_us(fn, n=10, reps=5):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(n):
            fn()
    gr.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        gr.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (reps * n) * 1e3


for shp in SHAPES:
    x = torch.randn(*shp, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    bn = nn.BatchNorm2d(shp[1]).to(dev)
    g = torch.randn_like(x)
    res = {}
    for fused in ("0", "1"):
        os.environ["PCOPS_BN_FUSED_FINAL"] = fused
        fwd = graph_us(lambda: bn_act(x, bn, ACT_RELU))
        both = graph_us(lambda: torch.autograd.grad(bn_act(x, bn, ACT_RELU), (x, bn.weight, bn.bias), g))
        res[fused] = (fwd, both - fwd)
    mb = x.numel() * 2 / 1e6
    print(f"{tag} {shp} {mb:.0f} MB: fwd unfused {res['0'][0]:.1f} us fused {res['1'][0]:.1f} us | "
          f"bwd unfused {res['0'][1]:.1f} us fused {res['1'][1]:.1f} us", flush=True)
