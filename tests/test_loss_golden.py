"""CD-L1 / loss parity against the REFERENCE's own loss code.

tests/golden/loss.npz was produced by tests/golden/make_golden_loss.py from
utils/loss_utils.py:33-155 (get_loss, get_loss_PM, calc_cd, calc_dcd) and
metrics/CD/fscore.py:3-16, with the Chamfer extension replaced by the
reference's own chamfer_python.distChamfer (float64) and fps_subsample's
CUDA ops by the build's FPS oracle.  The inputs are regenerated here from
the same numpy seeds (make_golden_loss.loss_case).

Bar (BASELINE.json north_star): Chamfer indices exact, values within 1e-5
abs.  Cases: configs[0] (B=4, N=2048) and the PCN shapes (B=2, 256 / 2048 /
16384 against a 16384-point gt).

  CPU  -- the package's metrics driven by oracle/cpu_path.py (C Chamfer
          restatement): pins the oracle to the reference's loss code.
  GPU  -- the package's metrics on libpcops (csrc/chamfer.hip, FPS, gather).
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden

sys.path.insert(0, GOLDEN)
from make_golden_loss import cases, loss_case  # noqa: E402

ATOL = 1e-5


def _run(name, dev):
    from svdformer_pointsea_amd import metrics as M

    pc, p1, p2, gt, partial = (torch.from_numpy(a).to(dev) for a in loss_case(*cases[name]))
    pred = (pc, p1, p2)
    res = {}
    for sq in (True, False):
        tag = "sqrt" if sq else "l2"
        tot, parts = M.get_loss(pred, gt, sqrt=sq)
        res[f"loss_{tag}"] = np.array([float(tot)] + [float(x) for x in parts])
        tot, parts = M.get_loss_PM(pred, partial, gt, sqrt=sq)
        res[f"losspm_{tag}"] = np.array([float(tot)] + [float(x) for x in parts])
    cd_p, cd_t, f1, d1, d2, i1, i2 = M.calc_cd(p2, gt, calc_f1=True, return_raw=True)
    res.update(cd_p=cd_p, cd_t=cd_t, f1=f1, d1=d1, d2=d2, i1=i1, i2=i2)
    sep = M.calc_cd(p2, gt, separate=True)
    res["sep_l1"], res["sep_l2"] = sep
    res["fscore"] = torch.stack(M.fscore(d1, d2))
    res["dcd"] = torch.stack(M.calc_dcd(p1, gt))
    res["dcd_nonreg"] = torch.stack(M.calc_dcd(p1, gt, non_reg=True))
    return {k: (v.detach().cpu().numpy() if torch.is_tensor(v) else v) for k, v in res.items()}


def _compare(name, res):
    ref = golden("loss.npz")
    for key in ("loss_sqrt", "loss_l2", "losspm_sqrt", "losspm_l2", "cd_p", "cd_t", "f1", "sep_l1", "sep_l2",
                "fscore", "dcd", "dcd_nonreg"):
        np.testing.assert_allclose(res[key], ref[f"{name}_{key}"], rtol=0, atol=ATOL, err_msg=f"{name} {key}")
    # the Chamfer nearest neighbours behind CD-L1 / DCD / F-score: exact
    np.testing.assert_array_equal(res["i1"], ref[f"{name}_i1"], err_msg=f"{name} idx1")
    np.testing.assert_array_equal(res["i2"], ref[f"{name}_i2"], err_msg=f"{name} idx2")
    if f"{name}_d1" in ref:
        np.testing.assert_allclose(res["d1"], ref[f"{name}_d1"], rtol=0, atol=ATOL)
        np.testing.assert_allclose(res["d2"], ref[f"{name}_d2"], rtol=0, atol=ATOL)
    # CD-L1 as test_pcn.py:63-66 reports it (x1e3): within 1e-5 of the reference too
    assert abs(float(res["cd_p"].mean()) * 1e3 - float(ref[f"{name}_cd_p"].mean()) * 1e3) < ATOL * 1e3


@pytest.mark.parametrize("name", ["c1", "pcn"])
def test_loss_golden_cpu_oracle(name):
    from oracle.cpu_path import cpu_ops

    with cpu_ops():
        res = _run(name, "cpu")
    _compare(name, res)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1", "pcn"])
def test_loss_golden_gpu(name, dev):
    _compare(name, _run(name, dev))
