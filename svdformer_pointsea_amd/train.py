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


def never_used(model):
    """Parameters the forward never reads: the BatchNorm of a Conv2d block
    built with if_bn=False (models/model_utils.py:27-43 constructs it anyway).
    The reference's per-tensor Adam/AdamW skips them (their .grad stays None);
    FlatParams keeps them out of the optimizer's segment to match."""
    names = set()
    for mname, m in model.named_modules():
        if getattr(m, "if_bn", True) is False and isinstance(getattr(m, "bn", None), nn.Module):
            for pname, _ in m.bn.named_parameters():
                names.add(f"{mname}.bn.{pname}" if mname else f"bn.{pname}")
    return names


class FlatParams:
    def __init__(self, model, device, bf16=True, frozen=None):
        self.model = model
        named = list(model.named_parameters())
        low = _bf16_names(model) if bf16 else set()
        frozen = never_used(model) if frozen is None else set(frozen)
        # layout: bf16-eligible | other trainable (fp32) | never-used (stable within each)
        named.sort(key=lambda kv: (kv[0] in frozen, kv[0] not in low))
        self.n16 = sum(p.numel() for n, p in named if n in low and n not in frozen)
        low = low - frozen
        total = sum(p.numel() for _, p in named)
        self.n_train = total - sum(p.numel() for n, p in named if n in frozen)
        self.frozen = frozen
        self.flat = torch.empty(total, dtype=torch.float32, device=device)
        # fp32 gradient bucket.  NOTE: after collect(widen=False) (the FlatAdam path) its shadow
        # slice [0, n16) is stale -- those gradients are in grad16 only; readers (grad norms,
        # clipping, finiteness checks) must read grad16 there
        self.grad = torch.zeros(total, dtype=torch.float32, device=device)
        self.flat16 = torch.empty(self.n16, dtype=torch.bfloat16, device=device)
        self.grad16 = torch.zeros(self.n16, dtype=torch.bfloat16, device=device)
        self.shadow = {}
        self._order = []   # bf16-eligible shadows in bucket order
        self._offset = {}  # parameter name -> offset in the flat buffers
        # with bf16 shadows (collect() required anyway) autograd also owns the fp32
        # parameters' gradients: a preset .grad view made AccumulateGrad launch one add
        # kernel per fp32 parameter per step (~90 LayerNorm / BatchNorm tensors, 0.45 ms
        # per PCN step); collect() gathers them with one batched copy instead
        self._own32 = bool(low) and _GRADS == "cat"
        self._order32 = []  # (parameter, its bucket view) of the trainable fp32 region
        off = 0
        with torch.no_grad():
            for name, p in named:
                n = p.numel()
                self._offset[name] = off
                view = self.flat[off:off + n].as_strided(p.shape, p.stride())
                view.copy_(p.data)
                p.data = view
                p.grad = self.grad[off:off + n].as_strided(p.shape, p.stride())
                if self._own32 and name not in low and name not in frozen:
                    self._order32.append((p, p.grad))
                if name in low:
                    w = self.flat16[off:off + n].as_strided(p.shape, p.stride())
                    w.requires_grad_(True)
                    if _GRADS == "preset":
                        w.grad = self.grad16[off:off + n].as_strided(p.shape, p.stride())
                    self.shadow[name] = w
                    self._order.append(w)
                off += n
        n32 = max((p.numel() for p, _ in self._order32), default=0)
        self._zeros32 = torch.zeros(n32, dtype=torch.float32, device=device)

    def master(self):
        """The whole fp32 master buffer as ONE parameter whose .grad is the bucket.
        Adam / AdamW are elementwise, so one update over the flat buffer equals
        the per-tensor updates when every parameter is in one param group with
        the same hyper-parameters (train_pcn.py:57-60, train_55.py:86-88), and
        the fused optimizer then runs one kernel over one tensor instead of
        chunking ~300 tensors (1.0 -> ~0.3 ms per PCN step).  Parameters the
        forward never reads sit at the end of the buffer and are left out, as
        the per-tensor optimizer skips them (AdamW would otherwise decay them)."""
        p = nn.Parameter(self.flat[:self.n_train])   # shares the storage; never-used tail excluded
        p.grad = self.grad[:self.n_train]
        return p

    def zero_grad(self):
        if self._own32:
            for p, _ in self._order32:
                p.grad = None          # grad[n16:n_train] is overwritten by collect()
        else:
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

    def collect(self, widen=True):
        """fp32 gradient bucket <- the shadows' bf16 gradients (zeros where a
        shadow received none): one batched concatenation, one cast kernel.
        widen=False leaves the shadow region in the bf16 bucket (grad16) for an
        optimizer that reads it there (FlatAdam); the fp32 region is gathered."""
        if not self._order:
            return
        with torch.no_grad():
            if _GRADS == "preset":
                if widen:
                    self.grad[:self.n16].copy_(self.grad16)
                return
            parts = []
            for w in self._order:
                g = w.grad
                parts.append(torch.zeros(w.numel(), dtype=self.grad16.dtype, device=self.grad16.device)
                             if g is None else self._physical(g, w))
            torch.cat(parts, out=self.grad16)
            if widen:
                self.grad[:self.n16].copy_(self.grad16)
            self._collect32(self.n16, self.n_train, self._order32)

    def _collect32(self, lo, hi, entries, stream=None):
        """bucket[lo:hi] <- the fp32 gradients autograd produced for `entries` (flat order),
        zeros where none arrived; .grad points at the bucket again afterwards.
        `stream`: the stream the gather runs on when it is not the one the
        gradients were produced on (they are recorded there before .grad lets go)."""
        if not self._own32 or not entries:
            return
        parts = []
        for p, view in entries:
            g = p.grad
            if g is not None and stream is not None:
                g.record_stream(stream)
            parts.append(self._zeros32[:p.numel()] if g is None else self._physical(g, p))
        torch.cat(parts, out=self.grad[lo:hi])
        for p, view in entries:
            p.grad = view

    def allreduce(self, world):
        """The data-parallel step's only collective: mean of the flat bucket."""
        if world > 1:
            import torch.distributed as dist
            dist.all_reduce(self.grad)
            self.grad.mul_(1.0 / world)


class FlatAdam:
    """`step()` of a torch Adam / AdamW over FlatParams.master() on libpcops (pcops_adam_flat): one
    pass that reads the shadow region's gradients from the bf16 bucket (collect(widen=False)), the
    rest from the fp32 bucket, updates master / exp_avg / exp_avg_sq in the torch optimizer's own
    state (so its state_dict, checkpoints and LR schedule are unchanged) and writes the new bf16
    shadow weights -- replacing the widening cast, torch's fused update and the shadow refresh.
    Arithmetic: torch's Adam (core/train_pcn.py:57-60 Adam, core/train_55.py:86-88 AdamW), the
    device step tensor incremented first as in torch's capturable path."""

    def __init__(self, opt, fp):
        if len(opt.param_groups) != 1 or len(opt.param_groups[0]["params"]) != 1:
            raise ValueError("FlatAdam: one param group holding FlatParams.master()")
        g = opt.param_groups[0]
        if g.get("amsgrad") or g.get("maximize") or g.get("differentiable"):
            raise ValueError("FlatAdam: amsgrad / maximize / differentiable are not used by the reference")
        self.opt, self.fp = opt, fp
        self.p = g["params"][0]
        if not self.p.is_cuda or self.p.dtype != torch.float32:
            raise ValueError("FlatAdam: the flat master must be an fp32 CUDA tensor")
        # torch >= 2.x: AdamW is Adam with decoupled_weight_decay=True, and plain Adam accepts the flag
        self.adamw = bool(g.get("decoupled_weight_decay", isinstance(opt, torch.optim.AdamW)))
        self._check_state()

    def _check_state(self):
        """The kernel dereferences the step counter and a tensor LR on the device: both must be
        0-dim fp32 tensors on the master's device.  A step kept as a Python number or a host /
        other-dtype tensor (a non-capturable optimizer, an old checkpoint) is converted here,
        eagerly; a tensor LR elsewhere is an error (the schedule writes it in place every step)."""
        p, g = self.p, self.opt.param_groups[0]
        lr = g["lr"]
        if isinstance(lr, torch.Tensor) and (lr.device != p.device or lr.dtype != torch.float32 or lr.dim() != 0):
            raise ValueError(f"FlatAdam: a tensor lr must be a 0-dim float32 tensor on {p.device} "
                             f"(got {lr.dtype} on {lr.device}, shape {tuple(lr.shape)})")
        st = self.opt.state.get(p)
        if not st:
            return
        step = st.get("step")
        if step is not None and not (isinstance(step, torch.Tensor) and step.device == p.device
                                     and step.dtype == torch.float32 and step.dim() == 0):
            st["step"] = torch.tensor(float(step), dtype=torch.float32, device=p.device)
        for k in ("exp_avg", "exp_avg_sq"):
            t = st.get(k)
            if t is None or t.device != p.device or t.dtype != torch.float32 or t.shape != p.shape \
                    or not t.is_contiguous():
                raise ValueError(f"FlatAdam: optimizer state {k!r} must be a contiguous fp32 tensor like the "
                                 f"master on {p.device}")

    @torch.no_grad()
    def step(self, bf16_grads=True):
        """bf16_grads: the shadow region's gradients are in fp.grad16 (collect(widen=False));
        False: the whole fp32 bucket (the data-parallel path's all-reduced gradients)."""
        from ._lib import call, lib, ptr, stream_of

        g = self.opt.param_groups[0]
        p = self.p
        st = self.opt.state[p]
        if not st:
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        elif not torch.cuda.is_current_stream_capturing():
            self._check_state()   # a state loaded since (load_state_dict) is validated before use
        st["step"].add_(1)
        # this IS the optimizer's step (its own step() is never called): flag it the way the LR
        # scheduler's wrapper of opt.step does, so the schedule does not take a batch_end() after
        # it for the "scheduler before optimizer" misuse (the LR sequence is pinned by
        # tests/test_train_flat.py::test_captured_flat_adam_follows_lr_schedule)
        self.opt._opt_called = True
        lr = g["lr"]
        lr_dev = lr if isinstance(lr, torch.Tensor) else None
        fp = self.fp
        beta1, beta2 = g["betas"]
        with torch.cuda.device(p.device):
            call("adam_flat", lib().pcops_adam_flat, ptr(p), ptr(fp.grad16) if bf16_grads else None, ptr(fp.grad),
                 fp.n16, p.numel(), ptr(st["exp_avg"]), ptr(st["exp_avg_sq"]), ptr(fp.flat16),
                 ptr(lr_dev), float(lr) if lr_dev is None else 0.0, ptr(st["step"]), float(beta1), float(beta2),
                 float(g["eps"]), float(g["weight_decay"]), int(self.adamw), stream_of(p))


class BucketedAllReduce:
    """The data-parallel gradient all-reduce, overlapped with backward.

    The flat gradient bucket is cut into contiguous buckets of ~bucket_mb MB
    (the bf16-eligible region from its END, since the backward pass produces
    the last layers' gradients first; the fp32 region as one bucket).  A
    post-accumulate-grad hook on every trainable parameter counts arrivals;
    when a bucket is complete its bf16 gradients are concatenated and widened
    into the fp32 bucket (as FlatParams.collect does for all of them at once)
    and its all-reduce is issued on a communication stream, while the compute
    stream carries on with the rest of the backward pass.  Buckets are issued
    strictly in bucket order (a ready bucket waits for its predecessors), so
    every rank issues the same collectives in the same order.  finish() issues
    whatever is left (parameters without a gradient contribute zeros) and
    makes the compute stream wait for the communication stream.

    Sum-then-scale per element, as FlatParams.allreduce: for two ranks the
    result is bitwise that of the single all-reduce (tests/test_ddp_gloo.py).
    Works eagerly and inside HIP-graph capture (the hooks run at capture
    time, so the captured graph holds the collectives)."""

    def __init__(self, fp, world, bucket_mb=25.0, group=None):
        import torch.distributed as dist

        self.fp, self.world, self.group, self.dist = fp, world, group, dist
        self.on_gpu = fp.flat.is_cuda
        self.comm = torch.cuda.Stream(device=fp.flat.device) if self.on_gpu else None
        # trainable entries in flat order: (offset, numel, tensor that receives the gradient)
        entries = []
        shadows = dict(fp.shadow)
        for n, p in sorted(fp.model.named_parameters(), key=lambda kv: fp._offset[kv[0]]):
            o = fp._offset[n]
            if n in fp.frozen:
                continue
            entries.append((o, p.numel(), shadows.get(n, p), n in shadows))
        per = max(1, int(bucket_mb * 2 ** 20 / 4))
        buckets = []   # (lo, hi, [entries]): contiguous, all bf16 shadows or all fp32 parameters
        for region in ([e for e in entries if e[3]], [e for e in entries if not e[3]]):
            cur, hi = [], None
            for e in reversed(region):                   # back to front: backward order
                if cur and hi - e[0] > per:
                    buckets.append((cur[-1][0], hi, cur))
                    cur, hi = [], None
                if hi is None:
                    hi = e[0] + e[1]
                cur.append(e)
            if cur:
                buckets.append((cur[-1][0], hi, cur))
        self.buckets = buckets
        self._bucket_of = {}
        for bi, (_, _, es) in enumerate(buckets):
            for e in es:
                self._bucket_of[id(e[2])] = bi
        self._hooks = []
        for _, _, es in buckets:
            for e in es:
                self._hooks.append(e[2].register_post_accumulate_grad_hook(self._arrived))
        self.reset()

    def reset(self):
        self._left = [len(es) for _, _, es in self.buckets]
        self._events = [[] for _ in self.buckets]
        self._next = 0

    def _arrived(self, t):
        bi = self._bucket_of.get(id(t))
        if bi is None:
            return
        if self.on_gpu:
            # the gradient was produced on the stream backward runs this node on
            # (the model's side-stream branches differentiate on their own
            # streams): the bucket's communication work waits for exactly that
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(t.device))
            self._events[bi].append(ev)
        self._left[bi] -= 1
        while self._next < len(self.buckets) and self._left[self._next] == 0:
            self._issue(self._next)
            self._next += 1

    def _issue(self, bi):
        lo, hi, es = self.buckets[bi]
        fp = self.fp
        if self.on_gpu:
            for ev in self._events[bi]:
                self.comm.wait_event(ev)
            with torch.cuda.stream(self.comm):
                self._reduce(lo, hi, es)
        else:
            self._reduce(lo, hi, es)

    def _reduce(self, lo, hi, es):
        fp = self.fp
        # the gradients were produced on the compute stream(s) and are read here on
        # the communication stream: each is recorded on it, so the allocator cannot
        # hand its block to the rest of backward before the gather below has run
        comm = self.comm if self.on_gpu else None
        with torch.no_grad():
            if es[0][3]:   # bf16 shadows: their gradients into the flat bf16 then the fp32 bucket
                if _GRADS != "preset":   # preset: the gradients already live in grad16[lo:hi]
                    parts = []
                    for o, n, w, _ in sorted(es, key=lambda e: e[0]):
                        g = w.grad
                        if g is not None and comm is not None:
                            g.record_stream(comm)
                        parts.append(torch.zeros(n, dtype=fp.grad16.dtype, device=fp.grad16.device)
                                     if g is None else fp._physical(g, w))
                    torch.cat(parts, out=fp.grad16[lo:hi])
                fp.grad[lo:hi].copy_(fp.grad16[lo:hi])
            elif fp._own32:   # fp32 parameters: autograd-owned gradients into the bucket
                view = {id(p): v for p, v in fp._order32}
                fp._collect32(lo, hi, [(w, view[id(w)]) for o, n, w, _ in sorted(es, key=lambda e: e[0])],
                              stream=comm)
            seg = fp.grad[lo:hi]
            self.dist.all_reduce(seg, group=self.group)
            seg.mul_(1.0 / self.world)

    def finish(self):
        """Issue the buckets still waiting (parameters that got no gradient) and
        join the communication stream; call after backward()."""
        if self.on_gpu and self._next < len(self.buckets):
            self.comm.wait_stream(torch.cuda.current_stream(self.fp.grad.device))
        while self._next < len(self.buckets):
            self._issue(self._next)
            self._next += 1
        if self.on_gpu:
            torch.cuda.current_stream(self.fp.grad.device).wait_stream(self.comm)
        self.reset()


# ------------------------------------------------------------------ LR schedules
class GradualWarmupScheduler(torch.optim.lr_scheduler.LRScheduler):
    """utils/schedular.py:5-64: linear warm-up of the learning rate over
    `total_epoch` scheduler steps (from 0 when multiplier == 1), then hand-off to
    `after_scheduler` (MultiStepLR for PCN, StepLR for ShapeNet-55), whose base
    LRs become base_lr * multiplier.  Same get_lr / step arithmetic as the
    reference; ReduceLROnPlateau hand-off is not used by either train loop and
    is not restated."""

    def __init__(self, optimizer, multiplier, total_epoch, after_scheduler=None):
        if multiplier < 1.0:
            raise ValueError("multiplier should be greater thant or equal to 1.")
        self.multiplier = multiplier
        self.total_epoch = total_epoch
        self.after_scheduler = after_scheduler
        self.finished = False
        super().__init__(optimizer)

    def get_lr(self):
        if self.last_epoch > self.total_epoch:
            if self.after_scheduler:
                if not self.finished:
                    self.after_scheduler.base_lrs = [b * self.multiplier for b in self.base_lrs]
                    self.finished = True
                return self.after_scheduler.get_last_lr()
            return [b * self.multiplier for b in self.base_lrs]
        if self.multiplier == 1.0:
            return [b * (float(self.last_epoch) / self.total_epoch) for b in self.base_lrs]
        return [b * ((self.multiplier - 1.0) * self.last_epoch / self.total_epoch + 1.0) for b in self.base_lrs]

    def step(self, epoch=None):
        if self.finished and self.after_scheduler:
            self.after_scheduler.step(None if epoch is None else epoch - self.total_epoch)
            self._last_lr = self.after_scheduler.get_last_lr()
        else:
            super().step(epoch)


class TrainSchedule:
    """The reference loops' LR policy around one optimizer
    (core/train_pcn.py:62-65,132-140; core/train_55.py:90-94,197-205):
    warm-up scheduler stepped once per batch for the first WARMUP_STEPS
    batches, then stepped once per epoch (MultiStepLR milestones / StepLR)."""

    def __init__(self, optimizer, model="svdformer", warmup_steps=300):
        from torch.optim.lr_scheduler import MultiStepLR, StepLR

        if model == "svdformer":   # config_pcn.py:70-73
            after = MultiStepLR(optimizer, milestones=[40, 80, 120, 160, 200, 240, 280, 320, 360], gamma=0.7)
        else:                      # config_55.py:70-72
            after = StepLR(optimizer, step_size=2, gamma=0.98)
        self.warmup_steps = warmup_steps
        self.sched = GradualWarmupScheduler(optimizer, multiplier=1, total_epoch=warmup_steps, after_scheduler=after)
        self.steps = 0

    def batch_end(self):
        if self.steps <= self.warmup_steps:
            self.sched.step()
            self.steps += 1

    def epoch_end(self):
        self.sched.step()

    def lr(self):
        v = self.sched.get_last_lr()[0]
        return float(v)


# ------------------------------------------------------------------ checkpoints
def checkpoint_state(model, optimizer, fp=None, prefix="module."):
    """The reference's checkpoint dict (core/train_pcn.py:152-166):
    {'model': state_dict with DataParallel's 'module.' prefix,
     'optimizer': the state_dict of a per-tensor Adam/AdamW over
                  model.parameters()}.
    With FlatParams the optimizer runs on one flat tensor; its moments are
    split back into per-parameter entries in model.parameters() order, and
    parameters the forward never reads get no entry (the per-tensor optimizer
    never creates state for a parameter whose .grad is None)."""
    sd = {prefix + k: v.detach().clone() for k, v in model.state_dict().items()}
    osd = optimizer.state_dict()
    if fp is None:
        return {"model": sd, "optimizer": osd}
    names = [n for n, _ in model.named_parameters()]
    params = dict(model.named_parameters())
    (flat_state,) = list(osd["state"].values()) or [{}]
    state = {}
    for i, n in enumerate(names):
        if n in fp.frozen or not flat_state:
            continue
        o, p = fp._offset[n], params[n]
        ent = {}
        for k, v in flat_state.items():
            if torch.is_tensor(v) and v.numel() == fp.n_train:
                ent[k] = v[o:o + p.numel()].view_as(p).clone()
            elif k == "step" and torch.is_tensor(v):
                # the per-tensor optimizer keeps its step as a host fp32 scalar
                ent[k] = v.detach().to("cpu", torch.float32).clone()
            else:
                ent[k] = v.clone() if torch.is_tensor(v) else v
        state[i] = ent
    (group,) = osd["param_groups"]
    return {"model": sd, "optimizer": {"state": state, "param_groups": [_reference_group(group, len(names))]}}


def _reference_group(group, nparams):
    """The flat optimizer's param_group as the reference's per-tensor Adam/AdamW
    writes it (core/train_pcn.py:57-60, core/train_55.py:86-88): host-float
    learning rates and the constructor defaults for the implementation
    switches the bench turns on (fused / capturable / foreach), so loading the
    checkpoint into torch.optim.Adam(model.parameters()) inherits none of them."""
    group = dict(group)
    for k in ("lr", "initial_lr"):
        if torch.is_tensor(group.get(k)):
            group[k] = float(group[k])
    group["fused"], group["capturable"], group["foreach"] = None, False, None
    group["params"] = list(range(nparams))
    return group


def load_checkpoint_state(ckpt, model, optimizer, fp=None, prefix="module."):
    """Inverse of checkpoint_state; also reads checkpoints written by the
    reference's per-tensor optimizer (the same layout)."""
    sd = {(k[len(prefix):] if k.startswith(prefix) else k): v for k, v in ckpt["model"].items()}
    model.load_state_dict(sd, strict=True)
    osd = ckpt["optimizer"]
    if fp is None:
        optimizer.load_state_dict(osd)
        return
    names = [n for n, _ in model.named_parameters()]
    params = dict(model.named_parameters())
    (group,) = osd["param_groups"]
    flat_state = {}
    for i, ent in osd["state"].items():
        n = names[int(i)]
        o, p = fp._offset[n], params[n]
        for k, v in ent.items():
            if torch.is_tensor(v) and v.shape == p.shape:
                buf = flat_state.setdefault(k, torch.zeros(fp.n_train, dtype=v.dtype, device=fp.flat.device))
                buf[o:o + p.numel()].view_as(p).copy_(v)
            else:
                flat_state[k] = v.clone() if torch.is_tensor(v) else v   # never alias the source's step
    (cur,) = optimizer.state_dict()["param_groups"]
    # the live optimizer's implementation switches win over the saved ones
    # (checkpoint_state writes the per-tensor defaults): a capturable / fused
    # flat optimizer stays one, and its step is placed on the device by
    # torch's loader because the group it sees says capturable
    group = {**group, "params": cur["params"]}
    for k in ("fused", "capturable", "foreach", "differentiable"):
        if k in cur:
            group[k] = cur[k]
    live = optimizer.param_groups[0]
    lr_tensors = {k: live[k] for k in ("lr", "initial_lr") if torch.is_tensor(live.get(k))}
    optimizer.load_state_dict({"state": {cur["params"][0]: flat_state} if flat_state else {},
                               "param_groups": [group]})
    # a captured graph reads the LR through the tensor it was captured with:
    # keep that tensor and write the saved value into it
    live = optimizer.param_groups[0]
    for k, t in lr_tensors.items():
        t.fill_(float(live[k]))
        live[k] = t
