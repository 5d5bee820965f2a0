"""kNN timing at the model shapes (HIP events); PCOPS_KNN_V1=1 selects the
first-generation feature-space kernel for A/B runs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svdformer_pointsea_amd.model_utils import _knn  # noqa: E402


def timeit(fn, iters=10, warm=2):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


dev = torch.device("cuda:0")
torch.manual_seed(0)
tag = "v1" if os.environ.get("PCOPS_KNN_V1") == "1" else "v2"
for (B, S, N, C, K, what) in [(32, 512, 2048, 3, 16, "sa1 query_knn"), (32, 2048, 2048, 3, 16, "gcn_1 self"),
                              (32, 512, 512, 64, 8, "svd gcn_2 self"), (16, 1024, 1024, 64, 8, "ps gcn_2 self"),
                              (16, 1024, 1024, 256, 4, "ps gcn_3 self")]:
    p = torch.randn(B, N, C, device=dev)
    q = p[:, :S].contiguous()
    ms = timeit(lambda: _knn(q, p, K), iters=10)
    fl = (2 * C + 2) * B * S * N
    print(f"{tag} {what}: B{B} S{S} N{N} C{C} K{K}: {ms:.3f} ms, {fl / ms / 1e9:.1f} TFLOP/s distance-equivalent",
          flush=True)
