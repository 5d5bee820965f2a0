"""Microbenchmark of the SVFNet image branch (ResNet-18, feature 16) and of
BatchNorm at its shapes, NCHW vs channels_last, under bf16 autocast."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from svdformer_pointsea_amd.svdformer import SVFNet, PCNConfig


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


dev = "cuda"
net = SVFNet(PCNConfig).img_feature_extractor.to(dev)
x = torch.rand(96, 1, 224, 224, device=dev)
for fmt in ["nchw", "cl"]:
    m = net.to(memory_format=torch.channels_last) if fmt == "cl" else net
    xi = x.to(memory_format=torch.channels_last) if fmt == "cl" else x

    def fb():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(xi)
        y.float().sum().backward()
    print(fmt, "img branch fwd+bwd ms", timeit(fb))
    for amp in [True]:
        def f():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = m(xi)
        print(fmt, "img branch fwd ms", timeit(f))

for shape in [(96, 16, 224, 224), (96, 32, 112, 112), (32, 32, 2048, 16)]:
    for dt in [torch.bfloat16, torch.float32]:
        for cl in [False, True]:
            a = torch.randn(shape, device=dev, dtype=dt, requires_grad=True)
            if cl:
                a = a.detach().to(memory_format=torch.channels_last).requires_grad_()
            w = torch.ones(shape[1], device=dev, requires_grad=True)
            b = torch.zeros(shape[1], device=dev, requires_grad=True)
            rm, rv = torch.zeros(shape[1], device=dev), torch.ones(shape[1], device=dev)
            g = torch.randn_like(a)

            def f():
                F.batch_norm(a, rm, rv, w, b, training=True)

            def fb():
                y = F.batch_norm(a, rm, rv, w, b, training=True)
                y.backward(g)
            print(shape, dt, "cl" if cl else "nchw", "bn fwd %.3f ms  fwd+bwd %.3f ms" % (timeit(f), timeit(fb)))
