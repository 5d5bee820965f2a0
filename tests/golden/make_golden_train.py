"""LR-schedule golden vectors from the REFERENCE's own scheduler
(utils/schedular.py:5-64 GradualWarmupScheduler) driven the way its train
loops drive it: stepped once per batch while steps <= WARMUP_STEPS, then once
per epoch (core/train_pcn.py:62-65,132-140 with MultiStepLR,
config_pcn.py:70-74; core/train_55.py:90-94,197-205 with StepLR,
config_55.py:68-72).  Build container only; writes tests/golden/lr_schedule.npz
(the learning rate after every batch, per policy).

    python tests/golden/make_golden_train.py
"""
import importlib.util
import os

import numpy as np
import torch
from torch.optim.lr_scheduler import MultiStepLR, StepLR

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
N_EPOCHS, N_BATCHES, WARMUP = 90, 7, 300   # 630 batches: warm-up ends inside epoch 43


def run(policy, GWS):
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], lr=1e-4)
    if policy == "pcn":
        after = MultiStepLR(opt, milestones=[40, 80, 120, 160, 200, 240, 280, 320, 360], gamma=0.7)
    else:
        after = StepLR(opt, step_size=2, gamma=0.98)
    sched = GWS(opt, multiplier=1, total_epoch=WARMUP, after_scheduler=after)
    steps, lrs = 0, []
    for _ in range(N_EPOCHS):
        for _ in range(N_BATCHES):
            lrs.append(opt.param_groups[0]["lr"])
            if steps <= WARMUP:
                sched.step()
                steps += 1
        sched.step()
    return np.array(lrs, np.float64)


def main():
    spec = importlib.util.spec_from_file_location("ref_schedular", os.path.join(REF, "utils/schedular.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = {p: run(p, mod.GradualWarmupScheduler) for p in ("pcn", "55")}
    np.savez_compressed(os.path.join(HERE, "lr_schedule.npz"), **out)
    print({k: (v.min(), v.max(), v[-1]) for k, v in out.items()})


if __name__ == "__main__":
    main()
