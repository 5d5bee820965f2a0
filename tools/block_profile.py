"""torch.profiler table of one SDG_Decoder (refine2.decoder2 shapes, B=32,
L=2048, 512 -> 1024) forward + backward under bf16 autocast."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile
from svdformer_pointsea_amd.attention import SDG_Decoder

torch.manual_seed(0)
dec = SDG_Decoder(512, 128, 8).cuda()
x = torch.randn(32, 512, 2048, device="cuda", requires_grad=True)


def step():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = dec(x)
    y.float().sum().backward()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CUDA, ProfilerActivity.CPU], record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=70,
                                                          max_name_column_width=45, max_shapes_column_width=110))
