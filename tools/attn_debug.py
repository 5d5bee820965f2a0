import math, sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svdformer_pointsea_amd.attention import attention_core
dev = torch.device("cuda:0")
def ref(q, k, v, H):
    Lq, B, E = q.shape; hd = E // H
    qq = q.double().reshape(Lq, B * H, hd).transpose(0, 1)
    kk = k.double().reshape(-1, B * H, hd).transpose(0, 1)
    vv = v.double().reshape(-1, B * H, hd).transpose(0, 1)
    o = torch.softmax(qq @ kk.transpose(1, 2) / math.sqrt(hd), -1) @ vv
    return o.transpose(0, 1).reshape(Lq, B, E)
torch.manual_seed(0)
for (Lq, Lk, D, qzero) in [(32, 32, 32, True), (32, 32, 32, False), (32, 64, 64, False), (3, 3, 64, False), (64, 32, 32, True)]:
    q = torch.randn(Lq, 1, D, device=dev)
    if qzero: q.zero_()
    k = torch.randn(Lk, 1, D, device=dev); v = torch.randn(Lk, 1, D, device=dev)
    for dt in (torch.float32, torch.bfloat16):
        o = attention_core(q.to(dt), k.to(dt), v.to(dt), 1).double()
        r = ref(q.to(dt).float(), k.to(dt).float(), v.to(dt).float(), 1)
        err = (o - r).abs()
        print(Lq, Lk, D, qzero, dt, 'maxerr', err.max().item(), 'worst (q,d)', divmod(err.reshape(Lq, -1).argmax().item(), D))
    if qzero:
        o = attention_core(q.bfloat16(), k.bfloat16(), v.bfloat16(), 1).float()
        print(' row0 ours', o[0, 0, :8].tolist()); print(' row0 ref ', ref(q.bfloat16().float(), k.bfloat16().float(), v.bfloat16().float(), 1)[0, 0, :8].tolist())
