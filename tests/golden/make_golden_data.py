"""Data-path golden vectors from the REFERENCE's own transforms and
normalisation (utils/data_transforms.py:153-245, utils/data_loaders.py:221-227),
in the build container only; writes tests/golden/data.npz.

cv2 / transforms3d / open3d / h5py are not installed: the modules are stubbed
for the import.  transforms3d.zooms.zfdir2mat (used by RandomMirrorPoints)
is given its published definition -- factor * I without a direction,
I + (factor - 1) d d^T along a unit direction d -- so the mirror vectors pin
the reference's composition logic, not transforms3d itself (unpinned).

Inputs come from numpy seeds stored beside the outputs; every transform is
run after np.random.seed(seed), as the tests replay it.

    python tests/golden/make_golden_data.py
"""
import importlib.util
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _stubs():
    sys.modules["cv2"] = types.ModuleType("cv2")
    t3 = types.ModuleType("transforms3d")
    zooms = types.ModuleType("transforms3d.zooms")

    def zfdir2mat(factor, direction=None):
        if direction is None:
            return np.eye(3) * factor
        d = np.asarray(direction, dtype=np.float64)
        d = d / np.linalg.norm(d)
        return np.eye(3) + (factor - 1.0) * np.outer(d, d)

    zooms.zfdir2mat = zfdir2mat
    t3.zooms = zooms
    t3.axangles = types.ModuleType("transforms3d.axangles")
    sys.modules["transforms3d"], sys.modules["transforms3d.zooms"] = t3, zooms
    sys.modules["transforms3d.axangles"] = t3.axangles


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    _stubs()
    dt = _load(os.path.join(REF, "utils/data_transforms.py"), "ref_data_transforms")
    out = {}
    for i, n in enumerate((500, 1024, 1500, 2048, 3000)):
        seed = 100 + i
        pc = np.random.default_rng(seed).random((n, 3)).astype(np.float32) - 0.5
        np.random.seed(seed)
        out[f"up_{n}"] = dt.UpSamplePoints({"n_points": 2048})(pc)
        np.random.seed(seed)
        out[f"rs_{n}"] = dt.RandomSamplePoints({"n_points": 2048})(pc)
    base = np.random.default_rng(7).random((64, 3)).astype(np.float32) - 0.5
    for r in (0.1, 0.3, 0.6, 0.9):
        out[f"mirror_{r}"] = dt.RandomMirrorPoints(None)(base.copy(), r)
    # pc_norm (data_loaders.py:221-227) as a plain function of the dataset class
    src = open(os.path.join(REF, "utils/data_loaders.py")).read()
    assert "def pc_norm(self, pc):" in src
    g = np.random.default_rng(9).random((4096, 3)).astype(np.float32) * 3 + 1
    ns = {"np": np}
    body = src[src.index("    def pc_norm(self, pc):"):src.index("    def __getitem__", src.index("def pc_norm"))]
    exec("class _D:\n" + body, ns)
    out["pcnorm_in_seed"] = np.array(9)
    out["pcnorm"] = ns["_D"]().pc_norm(g)
    np.savez_compressed(os.path.join(HERE, "data.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
