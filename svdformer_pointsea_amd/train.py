"""Train-step parameter storage for the bf16 step on MI355X.

The reference trains in fp32 (core/train_pcn.py); the bf16 build runs the
dense layers under torch.autocast.  Autocast casts every Linear / Conv
weight to bf16 at every use and casts each weight gradient back to fp32:
~300 + ~290 small cast launches per PCN step (~4 ms of a ~80 ms step).

FlatParams keeps the same numerics with three flat buffers instead:
  * every parameter is a view of ONE flat fp32 buffer (the optimizer's
    master weights) and its .grad a view of ONE flat fp32 gradient bucket
    (the single RCCL all-reduce of the data-parallel step);
  * the autocast-eligible parameters (Linear / Conv / MultiheadAttention
    weights and biases) come first, and their bf16 shadows are views of a
    flat bf16 buffer, refreshed by ONE cast kernel per step;
  * the model runs through torch.func.functional_call on the bf16 shadows, so
    autocast finds bf16 operands and casts nothing; autograd hands each shadow
    its gradient tensor (no pre-set .grad, so no accumulate-add per use: ~200
    tiny add kernels per PCN step), and collect() concatenates them in bucket
    order into a flat bf16 buffer and widens that into the fp32 bucket (a few
    batched-copy launches + ONE cast kernel).
Values are unchanged: under autocast those GEMMs/convs already read the
bf16-rounded weights and produce bf16 weight gradients that are then
widened, which is exactly what the two flat casts do.  Parameters outside
the eligible set (LayerNorm, BatchNorm) stay fp32 and get fp32 gradients
directly in the bucket.
"""
import os

import torch
from torch import nn

# A/B switch: "cat" (default) lets autograd own the shadows' gradients;
# "preset" pre-assigns them as views of the flat bf16 buffer (autograd then
# accumulates into them with one add kernel per use)
_GRADS = os.environ.get("PCOPS_FLATGRAD", "cat")

_ELIGIBLE = (nn.Linear, nn.Conv1d, nn.Conv2d, nn.ConvTranspose1d)


def _bf16_names(model):
    names = set()
    for mname, m in model.named_modules():
        if isinstance(m, _ELIGIBLE) or type(m).__name__ == "MultiheadAttention":
            for pname, _ in m.named_parameters(recurse=False):
                names.add(f"{mname}.{pname}" if mname else pname)
    return names


class FlatParams:
    def __init__(self, model, device, bf16=True):
        self.model = model
        named = list(model.named_parameters())
        low = _bf16_names(model) if bf16 else set()
        named.sort(key=lambda kv: kv[0] not in low)          # bf16-eligible first (stable)
        self.n16 = sum(p.numel() for n, p in named if n in low)
        total = sum(p.numel() for _, p in named)
        self.flat = torch.empty(total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(total, dtype=torch.float32, device=device)
        self.flat16 = torch.empty(self.n16, dtype=torch.bfloat16, device=device)
        self.grad16 = torch.zeros(self.n16, dtype=torch.bfloat16, device=device)
        self.shadow = {}
        self._order = []   # bf16-eligible shadows in bucket order
        off = 0
        with torch.no_grad():
            for name, p in named:
                n = p.numel()
                view = self.flat[off:off + n].as_strided(p.shape, p.stride())
                view.copy_(p.data)
                p.data = view
                p.grad = self.grad[off:off + n].as_strided(p.shape, p.stride())
                if name in low:
                    w = self.flat16[off:off + n].as_strided(p.shape, p.stride())
                    w.requires_grad_(True)
                    if _GRADS == "preset":
                        w.grad = self.grad16[off:off + n].as_strided(p.shape, p.stride())
                    self.shadow[name] = w
                    self._order.append(w)
                off += n

    def master(self):
        """The whole fp32 master buffer as ONE parameter whose .grad is the bucket.
        Adam / AdamW are elementwise, so one update over the flat buffer equals
        the per-tensor updates when every parameter is in one param group with
        the same hyper-parameters (train_pcn.py:57-60, train_55.py:86-88), and
        the fused optimizer then runs one kernel over one tensor instead of
        chunking ~300 tensors (1.0 -> ~0.3 ms per PCN step)."""
        p = nn.Parameter(self.flat)   # shares the storage
        p.grad = self.grad
        return p

    def zero_grad(self):
        self.grad[self.n16:].zero_()   # grad[:n16] is overwritten by collect()
        if _GRADS == "preset":
            self.grad16.zero_()
            return
        for w in self._order:
            w.grad = None

    def refresh(self):
        """bf16 shadows <- fp32 master weights (one cast kernel)."""
        with torch.no_grad():
            self.flat16.copy_(self.flat[:self.n16])

    def forward(self, *args, **kwargs):
        """model(*args) on the bf16 shadows (falls back to the module when bf16=False)."""
        if not self.shadow:
            return self.model(*args, **kwargs)
        return torch.func.functional_call(self.model, self.shadow, args, kwargs, strict=False)

    @staticmethod
    def _physical(g, w):
        """g's elements in w's memory order, as a 1-D tensor (w is a dense view)."""
        if g.stride() != w.stride():
            h = torch.empty_strided(w.shape, w.stride(), dtype=g.dtype, device=g.device)
            h.copy_(g)
            g = h
        return g.as_strided((g.numel(),), (1,), g.storage_offset())

    def collect(self):
        """fp32 gradient bucket <- the shadows' bf16 gradients (zeros where a
        shadow received none): one batched concatenation, one cast kernel."""
        if not self._order:
            return
        with torch.no_grad():
            if _GRADS == "preset":
                self.grad[:self.n16].copy_(self.grad16)
                return
            parts = []
            for w in self._order:
                g = w.grad
                parts.append(torch.zeros(w.numel(), dtype=self.grad16.dtype, device=self.grad16.device)
                             if g is None else self._physical(g, w))
            torch.cat(parts, out=self.grad16)
            self.grad[:self.n16].copy_(self.grad16)

    def allreduce(self, world):
        """The data-parallel step's only collective: mean of the flat bucket."""
        if world > 1:
            import torch.distributed as dist
            dist.all_reduce(self.grad)
            self.grad.mul_(1.0 / world)
