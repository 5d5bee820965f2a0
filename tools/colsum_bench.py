"""pcops_colsum timing at the PCN bias-gradient shapes (HIP events, mean of 50):
achieved HBM rate of the (rows, C) bf16 read (eager: small shapes measure the host issue rate).  Knobs by env (PCOPS_COLSUM_BLOCKS,
PCOPS_COLSUM_CHUNKS) for A/B runs.

    python tools/colsum_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from svdformer_pointsea_amd.attention import colsum

SHAPES = [(65536, 1024), (65536, 512), (16384, 768), (16384, 512), (65536, 128), (1048576, 32), (524288, 128)]
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("PCOPS_COLSUM")) or "default"
dev = torch.device("cuda", 0)
for rows, C in SHAPES:
    g = torch.randn(rows, C, device=dev).to(torch.bfloat16)
    ref = g.double().sum(0)
    out = colsum(g, out_dtype=torch.float32)
    err = ((out.double() - ref).abs() / (g.double().abs().sum(0) + 1e-9)).max().item()
    for _ in range(5):
        colsum(g, out_dtype=torch.float32)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        colsum(g, out_dtype=torch.float32)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    print(f"{tag}: rows={rows} C={C} {us:7.1f} us {rows * C * 2 / us / 1e6:6.2f} TB/s relerr={err:.1e}", flush=True)
