"""Bias-gradient column sum: pcops_colsum vs torch's g.sum(0) at the PCN
shapes, 20 calls captured in a HIP graph (no host launch cost), replay timed
with events.  PCOPS_COLSUM_BLOCKS / PCOPS_COLSUM_CHUNKS select the pcops
launch shape (A/B)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from svdformer_pointsea_amd import attention

tag = f"blocks={os.environ.get('PCOPS_COLSUM_BLOCKS', 'dflt')} chunks={os.environ.get('PCOPS_COLSUM_CHUNKS', 'dflt')}"
fns = {"torch": lambda g: g.sum(0), "pcops": attention.colsum}
which = sys.argv[1:] or list(fns)
for rows, C in [(65536, 512), (65536, 1024), (65536, 256), (65536, 128), (16384, 512), (8192, 1024), (65536, 64)]:
    g = torch.randn(rows, C, device="cuda", dtype=torch.bfloat16)
    res = []
    for name in which:
        fn = fns[name]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                fn(g)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(20):
                fn(g)
        graph.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            graph.replay()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / 100 * 1e3
        res.append(f"{name} {us:.1f} us ({rows * C * 2 / us / 1e3:.0f} GB/s)")
    print(f"[{tag}] rows={rows} C={C}: " + " | ".join(res), flush=True)
