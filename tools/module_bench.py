"""Per-submodule fwd+bwd time of the PCN step (bf16 autocast, B=32): captures
each top-level submodule's inputs from one model forward, then times the
submodule alone (forward + backward of sum of outputs)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bench import synth_pcn
from svdformer_pointsea_amd.render import PCViews
from svdformer_pointsea_amd.svdformer import Model, PCNConfig, get_loss

dev = torch.device("cuda", 0)
if os.environ.get("BENCHMARK") == "1":
    torch.backends.cudnn.benchmark = True
torch.manual_seed(0)
model = Model(PCNConfig).to(dev)
partial, gt = synth_pcn(32, 1000, dev)
render = PCViews(TRANS=-0.7, RESOLUTION=224)
depth = render.get_img(partial).unsqueeze(1)
targets = {
    "encoder": model.encoder, "encoder.point_feature_extractor": model.encoder.point_feature_extractor,
    "encoder.img_feature_extractor": model.encoder.img_feature_extractor, "encoder.sa": model.encoder.sa,
    "encoder.viewattn": model.encoder.viewattn, "localencoder": model.localencoder, "refine1": model.refine1,
    "refine2": model.refine2, "refine2.sa1": model.refine2.sa1, "refine2.decoder1": model.refine2.decoder1,
    "refine2.cross1": model.refine2.cross1, "refine2.decoder2": model.refine2.decoder2,
    "refine1.decoder1": model.refine1.decoder1}
caught = {}
hooks = [m.register_forward_hook(lambda m, i, o, n=n: (caught.setdefault(n, i), None)[1]) for n, m in targets.items()]
with torch.autocast("cuda", dtype=torch.bfloat16):
    model(partial, depth)
for h in hooks:
    h.remove()


def run(mod, inp):
    inp = [x.detach().requires_grad_(x.is_floating_point()) if torch.is_tensor(x) else x for x in inp]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = mod(*inp)
    outs = out if isinstance(out, (tuple, list)) else (out,)
    s = sum(o.float().sum() for o in outs if torch.is_tensor(o) and o.is_floating_point())
    s.backward()


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


for n, m in targets.items():
    print(f"{n:40s} {timeit(lambda: run(m, caught[n])):8.2f} ms", flush=True)


def loss_only():
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        pc = model(partial, depth)
    pc = [p.detach().requires_grad_() for p in pc]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss, _ = get_loss(pc, gt)
    loss.backward()


print(f"{'get_loss (+ fwd no-grad)':40s} {timeit(loss_only):8.2f} ms")
opt = torch.optim.Adam(model.parameters(), lr=1e-4, fused=True)
for p in model.parameters():
    p.grad = torch.zeros_like(p)
print(f"{'adam fused step':40s} {timeit(opt.step):8.2f} ms")
