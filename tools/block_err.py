"""Where a block's fp32 error comes from (GPU): the refine2 blocks of
tests/golden/make_golden_attn_large.py run in float64 with ONE stage at a
time dropped to fp32 on the GPU, each reported as the max abs error of the
block output against the all-float64 run.  Stages: the 1x1 input conv
(MIOpen / GEMM), the q/k/v / out projections + FFN linears (hipBLASLt), the
attention core (libpcops exact-f32 MFMA), the LayerNorms (libpcops), and
all of them together (== the fp32 block).  The stage runner is the one
tests/test_gpu_attention.py::test_blocks_large_golden asserts with.

    python tools/block_err.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
from test_gpu_attention import LARGE, _stage_run  # noqa: E402


def main():
    torch.set_grad_enabled(False)
    dev = torch.device("cuda:0")
    for name in LARGE:
        exact = _stage_run(name, dev, ())
        row = []
        for st in [("conv",), ("linear",), ("core",), ("layernorm",), ("conv", "linear", "core", "layernorm")]:
            e = (_stage_run(name, dev, st) - exact).abs().max().item()
            row.append(f"{'+'.join(st) if len(st) < 4 else 'all'}={e:.2e}")
        print(name, " ".join(row), flush=True)


if __name__ == "__main__":
    main()
