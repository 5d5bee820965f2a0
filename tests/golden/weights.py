"""Deterministic, platform-independent parameter fill shared by the golden
generator (which loads it into the reference's modules) and the tests (which
load it into this package's mirror modules).  Only numpy's PCG64 stream is
used, so nothing but the seed needs to be committed."""
import numpy as np


def fill_state(module, seed, scale=0.05):
    """Overwrite every parameter/buffer of `module` in sorted-key order."""
    import torch

    rng = np.random.default_rng(seed)
    sd = module.state_dict()
    new = {}
    for key in sorted(sd):
        t = sd[key]
        if not torch.is_floating_point(t):
            new[key] = t
            continue
        shape = tuple(t.shape)
        if key.endswith("norm12.weight") or key.endswith("norm13.weight"):
            v = 1.0 + 0.1 * rng.standard_normal(shape)
        elif key.endswith("running_var"):  # BatchNorm eval statistics must stay positive
            v = 1.0 + 0.1 * np.abs(rng.standard_normal(shape))
        else:
            v = scale * rng.standard_normal(shape)
        new[key] = torch.from_numpy(v.astype(np.float32))
    module.load_state_dict(new)
    return module
