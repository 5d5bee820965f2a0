"""Data path (svdformer_pointsea_amd/datasets.py) against golden vectors from
the reference's own transforms (tests/golden/make_golden_data.py) and PCD
round trips.  CPU only."""
import numpy as np
import pytest
import torch

from conftest import golden
from svdformer_pointsea_amd import datasets as D


@pytest.mark.parametrize("n", [500, 1024, 1500, 2048, 3000])
def test_upsample_and_random_sample_match_reference(n):
    g = golden("data.npz")
    pc = np.random.default_rng(100 + [500, 1024, 1500, 2048, 3000].index(n)).random((n, 3)).astype(np.float32) - 0.5
    np.random.seed(100 + [500, 1024, 1500, 2048, 3000].index(n))
    up = D.UpSamplePoints({"n_points": 2048})(pc)
    np.testing.assert_array_equal(up, g[f"up_{n}"])
    np.random.seed(100 + [500, 1024, 1500, 2048, 3000].index(n))
    np.testing.assert_array_equal(D.RandomSamplePoints({"n_points": 2048})(pc), g[f"rs_{n}"])
    if n <= 2048:   # up-sampling keeps every original point and only duplicates them
        assert set(map(tuple, up.tolist())) == set(map(tuple, pc.tolist()))


@pytest.mark.parametrize("r", [0.1, 0.3, 0.6, 0.9])
def test_mirror_matches_reference(r):
    g = golden("data.npz")
    base = np.random.default_rng(7).random((64, 3)).astype(np.float32) - 0.5
    np.testing.assert_array_equal(D.RandomMirrorPoints()(base.copy(), r), g[f"mirror_{r}"])


def test_pc_norm_matches_reference():
    g = golden("data.npz")
    x = np.random.default_rng(int(g["pcnorm_in_seed"])).random((4096, 3)).astype(np.float32) * 3 + 1
    y = D.pc_norm(x)
    np.testing.assert_array_equal(y, g["pcnorm"])
    assert abs(np.sqrt((y ** 2).sum(1)).max() - 1.0) < 1e-6


@pytest.mark.parametrize("binary", [False, True])
def test_pcd_round_trip_and_io_dispatch(tmp_path, binary):
    rng = np.random.default_rng(3)
    pts = (rng.random((1000, 3)) - 0.5).astype(np.float32)
    path = str(tmp_path / "x.pcd")
    D.write_pcd(path, pts, binary=binary)
    back = D.IO.get(path)
    assert back.shape == (1000, 3) and back.dtype == np.float64
    np.testing.assert_array_equal(back.astype(np.float32), pts)
    np.save(str(tmp_path / "y.npy"), pts)
    np.testing.assert_array_equal(D.IO.get(str(tmp_path / "y.npy")), pts)


def test_pcd_reader_fields_and_refusals(tmp_path):
    """Extra fields (rgb, intensity), COUNT > 1, non-finite rows dropped (as
    open3d does); binary_compressed refused (utils/io.py supports
    uncompressed PCD only)."""
    path = tmp_path / "f.pcd"
    rows = "1 2 3 0.5 7 8\n4 5 6 0.25 9 10\nnan 0 0 1 1 1\n"
    path.write_text("VERSION 0.7\nFIELDS x y z intensity n\nSIZE 4 4 4 4 4\nTYPE F F F F F\nCOUNT 1 1 1 1 2\n"
                    "WIDTH 3\nHEIGHT 1\nPOINTS 3\nDATA ascii\n" + rows)
    np.testing.assert_array_equal(D.read_pcd(str(path)), [[1, 2, 3], [4, 5, 6]])
    bad = tmp_path / "c.pcd"
    bad.write_bytes(b"VERSION 0.7\nFIELDS x y z\nSIZE 4 4 4\nTYPE F F F\nCOUNT 1 1 1\nWIDTH 1\nHEIGHT 1\n"
                    b"POINTS 1\nDATA binary_compressed\n\x00\x00")
    with pytest.raises(ValueError):
        D.read_pcd(str(bad))


def test_pcn_pipeline_and_collate():
    """The train pipeline of data_loaders.py:136-151 on one sample, then the
    collate into the (B, 2048, 3) / (B, 16384, 3) batch the step consumes."""
    rng = np.random.default_rng(4)
    batch = []
    for i in range(3):
        data = {"partial_cloud": (rng.random((900 + i, 3)) - 0.5).astype(np.float32),
                "gtcloud": (rng.random((16384, 3)) - 0.5).astype(np.float32)}
        np.random.seed(i)
        out = D.pcn_train_transforms()(data)
        batch.append(("02691156", f"m{i}", out))
    tax, mids, data = D.collate(batch)
    assert data["partial_cloud"].shape == (3, 2048, 3) and data["gtcloud"].shape == (3, 16384, 3)
    assert data["partial_cloud"].dtype == torch.float32 and mids == ["m0", "m1", "m2"]
