"""EMD auction (metrics/EMD) on libpcops vs the oracle's deterministic restatement."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from svdformer_pointsea_amd.emd_module import emd_raw, emdModule

pytestmark = pytest.mark.gpu


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("B,n,eps,iters", [(2, 1024, 0.005, 50), (1, 1024, 0.05, 200), (3, 100, 0.005, 30),
                                           (1, 1, 0.005, 3), (2, 257, 0.002, 1)])
def test_emd_matches_oracle(dev, B, n, eps, iters):
    rng = np.random.default_rng(n + iters)
    x1 = (rng.random((B, n, 3)) - 0.5).astype(np.float32)
    x2 = (rng.random((B, n, 3)) - 0.5).astype(np.float32)
    d, a = emd_raw(T(x1, dev), T(x2, dev), eps, iters)
    rd, ra = O.emd(x1, x2, eps, iters)
    np.testing.assert_array_equal(a.cpu().numpy(), ra)
    np.testing.assert_array_equal(d.cpu().numpy(), rd)


def test_emd_ties_duplicate_points(dev):
    rng = np.random.default_rng(5)
    base = (rng.random((1, 256, 3)) - 0.5).astype(np.float32)
    x1 = np.tile(base, (1, 4, 1))          # every point 4 times -> equal bids
    x2 = np.tile(base[:, ::-1], (1, 4, 1)).copy()
    d, a = emd_raw(T(x1, dev), T(x2, dev), 0.005, 40)
    rd, ra = O.emd(x1, x2, 0.005, 40)
    np.testing.assert_array_equal(a.cpu().numpy(), ra)
    np.testing.assert_array_equal(d.cpu().numpy(), rd)


def test_emd_module_and_backward(dev):
    rng = np.random.default_rng(9)
    x1 = T((rng.random((2, 2048, 3)) - 0.5).astype(np.float32), dev).requires_grad_()
    x2 = T((rng.random((2, 2048, 3)) - 0.5).astype(np.float32), dev)
    dist, ass = emdModule()(x1, x2, 0.005, 50)
    g = torch.rand_like(dist)
    dist.backward(g)
    a = ass.long()
    assert (a >= 0).all()
    # CalcDist / NmDistanceGradKernel semantics
    matched = torch.gather(x2, 1, a[..., None].expand(-1, -1, 3))
    torch.testing.assert_close(dist, ((x1.detach() - matched) ** 2).sum(-1), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(x1.grad, 2 * g[..., None] * (x1.detach() - matched), rtol=1e-6, atol=1e-7)
    rg = O.emd_backward(x1.detach().cpu().numpy(), x2.cpu().numpy(), g.cpu().numpy(), ass.cpu().numpy())
    np.testing.assert_array_equal(x1.grad.cpu().numpy(), rg)


def test_emd_converges_full_size(dev):
    # size-independent property at a PCN-sized cloud: with enough iterations
    # the auction is a bijection and identical clouds map to themselves
    rng = np.random.default_rng(3)
    x = T((rng.random((4, 8192, 3)) - 0.5).astype(np.float32), dev)
    d, a = emd_raw(x, x.clone(), 0.005, 60)
    assert (a.long() == torch.arange(8192, device=dev)).float().mean() > 0.99
    assert d.max().item() < 1e-2


def test_emd_errors(dev):
    x = torch.rand(1, 1000, 3, device=dev)
    with pytest.raises(RuntimeError, match="multiple of 1024"):
        emdModule()(x, x, 0.005, 10)
    with pytest.raises(AssertionError):
        emdModule()(torch.rand(1, 1024, 3, device=dev), torch.rand(1, 2048, 3, device=dev), 0.005, 10)
