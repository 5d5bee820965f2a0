"""torch.profiler view of one bench step (op-level attribution of the torch
glue around libpcops): python tools/step_profile.py [--batch 32]"""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile

from bench import synth_pcn
from svdformer_pointsea_amd.render import PCViews
from svdformer_pointsea_amd.svdformer import Model, PCNConfig, get_loss

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--rows", type=int, default=60)
args = ap.parse_args()
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = Model(PCNConfig).to(dev)
opt = torch.optim.Adam(model.parameters(), lr=1e-4, fused=True)
render = PCViews(TRANS=-0.7, RESOLUTION=224)
partial, gt = synth_pcn(args.batch, 1000, dev)


def step():
    depth = render.get_img(partial).unsqueeze(1)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss, _ = get_loss(model(partial, depth), gt)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=args.rows, max_name_column_width=60))
print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=args.rows,
                                                          max_name_column_width=40, max_shapes_column_width=90))
