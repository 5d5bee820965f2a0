"""FPS launch times (HIP events) at the step's shapes, B = 32: us per round.
PCOPS_FPS_WAVE=0 in the environment keeps small clouds on the 8-wave block kernel (A/B)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from svdformer_pointsea_amd.pointnet2_utils import furthest_point_sample  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device="cpu").manual_seed(0)
tag = "wave=" + os.environ.get("PCOPS_FPS_WAVE", "8") + " mw=" + os.environ.get("PCOPS_FPS_MW", "0")
for B, N, M, kind in [(32, 16384, 2048, "gauss"), (32, 16384, 2048, "surface"), (16, 8192, 2048, "surface"),
                      (32, 2304, 512, "surface"), (16, 2304, 1024, "surface"), (32, 4096, 1024, "gauss"), (32, 2048, 512, "gauss"),
                      (32, 2048, 256, "gauss"), (32, 512, 128, "gauss"), (32, 1024, 256, "gauss")]:
    x = torch.randn(B, N, 3, generator=g)
    if kind == "surface":  # points on ellipsoid surfaces, like the PCN / ShapeNet gt clouds
        x = x / x.norm(dim=-1, keepdim=True) * torch.tensor([0.4, 0.25, 0.15])
    x = (x * 0.45 if kind == "gauss" else x).contiguous().to(dev)
    for _ in range(2):
        furthest_point_sample(x, M)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        furthest_point_sample(x, M)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(f"{tag} B={B} {N}->{M} {kind}: {ms:.3f} ms  {ms * 1e3 / (M - 1):.3f} us/round", flush=True)
