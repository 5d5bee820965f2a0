"""The package's SVDFormer / PointSea restatements against the reference's own
model code (tests/golden/make_golden_models.py): same state_dict keys and
shapes (reference checkpoints load strictly), and the same eval-mode forward
on the same weights and inputs.  CPU: the point ops run through the oracle
(oracle/cpu_path.py), exactly the stand-ins the generator gave the reference;
the GPU variants run libpcops (tests/test_gpu_model.py style tolerance)."""
import numpy as np
import pytest
import torch

import os
import sys

from conftest import golden

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from weights import fill_state  # noqa: E402
from make_golden_models import PCN, S55, SEED_PS, SEED_SVD  # noqa: E402
from oracle.cpu_path import cpu_ops, depth_images, real_images  # noqa: E402
from svdformer_pointsea_amd import pointsea, svdformer  # noqa: E402
from svdformer_pointsea_amd.render import PCViews, PCViews_Real  # noqa: E402

G = golden("models.npz")


def _build(which):
    if which == "svd":
        return fill_state(svdformer.Model(svdformer.PCNConfig), SEED_SVD).eval()
    return fill_state(pointsea.Model(pointsea.Config55), SEED_PS).eval()


@pytest.mark.parametrize("which", ["svd", "ps"])
def test_state_dict_matches_reference(which):
    sd = _build(which).state_dict()
    keys = sorted(sd)
    assert keys == list(G[f"{which}_keys"])
    assert [str(tuple(sd[k].shape)) for k in keys] == list(G[f"{which}_shapes"])


def _images(which, x, cpu):
    if which == "svd":
        r = PCViews(TRANS=-PCN["view_distance"], RESOLUTION=224)
        return depth_images(r, x).unsqueeze(1) if cpu else r.get_img(x).unsqueeze(1)
    r = PCViews_Real(TRANS=-S55["view_distance"])
    return real_images(r, x) if cpu else r.get_img(x)


@pytest.mark.parametrize("which", ["svd", "ps"])
def test_forward_matches_reference_cpu(which):
    m = _build(which)
    x = torch.from_numpy(G[f"{which}_partial"])
    with torch.no_grad(), cpu_ops():
        out = m(x, _images(which, x, True))
    for i, o in enumerate(out):
        ref = G[f"{which}_out{i}"]
        assert o.shape == ref.shape
        # same CPU torch underneath; only the token-major GEMM summation order differs
        np.testing.assert_allclose(o.numpy(), ref, rtol=0, atol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["svd", "ps"])
def test_forward_matches_reference_gpu(dev, which):
    m = _build(which).to(dev)
    x = torch.from_numpy(G[f"{which}_partial"]).to(dev)
    with torch.no_grad():
        out = m(x, _images(which, x, False))
    for i, o in enumerate(out):
        # dense layers round differently on the GPU (hipBLASLt / MIOpen); outputs are O(0.5)
        np.testing.assert_allclose(o.cpu().numpy(), G[f"{which}_out{i}"], rtol=0, atol=2e-3)
