"""Host-side data path of the reference's loaders, without open3d / cv2 /
transforms3d (absent here): point-cloud file I/O, the PCN transforms that
shape the hot path's inputs, and ShapeNet-55 normalisation.

  IO.get(path)              utils/io.py:27-48 dispatch by extension
                            (.pcd, .npy, .h5 / .txt)
  read_pcd / write_pcd      utils/io.py:97-115 (open3d.io.read_point_cloud):
                            PCD v0.7 'DATA ascii' and 'DATA binary'; like the
                            reference ("Support PCD files without compression
                            ONLY!"), binary_compressed is refused
  UpSamplePoints            utils/data_transforms.py:153-172 (tiles the cloud
                            up to n_points -- the exact duplicates FPS / kNN /
                            Chamfer tie rules are tested on)
  RandomSamplePoints        :175-187
  RandomMirrorPoints        :228-245 (x / z / xz mirror by a uniform draw)
  ScalePoints               :213-226
  pc_norm                   utils/data_loaders.py:221-227 (ShapeNet-55)
  collate                   utils/data_loaders.py:32-45 (stack the dict items)

Every transform draws from numpy's global RNG exactly as the reference does,
so seeded runs reproduce the reference's outputs (tests/test_datasets.py,
golden vectors from the reference's own transforms).
"""
import os

import numpy as np
import torch


# ------------------------------------------------------------------ PCD files
_PCD_NP = {("F", 4): np.float32, ("F", 8): np.float64, ("I", 1): np.int8, ("I", 2): np.int16,
           ("I", 4): np.int32, ("I", 8): np.int64, ("U", 1): np.uint8, ("U", 2): np.uint16,
           ("U", 4): np.uint32, ("U", 8): np.uint64}


def _pcd_header(f):
    meta, lines = {}, 0
    while True:
        raw = f.readline()
        if not raw:
            raise ValueError("PCD: missing DATA line")
        lines += 1
        line = raw.decode("ascii", "replace").strip()
        if not line or line.startswith("#"):
            continue
        key, *vals = line.split()
        meta[key.upper()] = vals
        if key.upper() == "DATA":
            return meta


def read_pcd(path):
    """(N, 3) float64 xyz of a PCD file, as open3d.io.read_point_cloud(...).points."""
    with open(path, "rb") as f:
        meta = _pcd_header(f)
        fields = [x.lower() for x in meta["FIELDS"]]
        sizes = [int(x) for x in meta.get("SIZE", ["4"] * len(fields))]
        types = [x.upper() for x in meta.get("TYPE", ["F"] * len(fields))]
        counts = [int(x) for x in meta.get("COUNT", ["1"] * len(fields))]
        n = int(meta["POINTS"][0]) if "POINTS" in meta else int(meta["WIDTH"][0]) * int(meta.get("HEIGHT", ["1"])[0])
        kind = meta["DATA"][0].lower()
        cols = []
        for name, c in zip(fields, counts):
            cols += [name] if c == 1 else [f"{name}{i}" for i in range(c)]
        if kind == "ascii":
            body = f.read().decode("ascii", "replace").split()
            vals = np.array(body[:n * len(cols)], dtype=np.float64).reshape(n, len(cols)) if n else np.zeros((0, len(cols)))
            table = {c: vals[:, i] for i, c in enumerate(cols)}
        elif kind == "binary":
            dt = np.dtype([(c, _PCD_NP[(t, s)]) for name, s, t, cnt in zip(fields, sizes, types, counts)
                           for c in ([name] if cnt == 1 else [f"{name}{i}" for i in range(cnt)])])
            rec = np.frombuffer(f.read(dt.itemsize * n), dtype=dt, count=n)
            table = {c: rec[c].astype(np.float64) for c in cols}
        else:
            raise ValueError(f"PCD: DATA {kind} not supported (uncompressed ascii / binary only)")
    pts = np.stack([table["x"], table["y"], table["z"]], axis=1)
    return pts[np.isfinite(pts).all(axis=1)]   # open3d drops non-finite points


def write_pcd(path, points, binary=False):
    """Write (N, 3) xyz as a PCD v0.7 file (float32 fields x y z)."""
    points = np.asarray(points, dtype=np.float32).reshape(-1, 3)
    n = points.shape[0]
    head = ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z\nSIZE 4 4 4\nTYPE F F F\n"
            f"COUNT 1 1 1\nWIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\n"
            f"DATA {'binary' if binary else 'ascii'}\n")
    with open(path, "wb") as f:
        f.write(head.encode("ascii"))
        if binary:
            f.write(np.ascontiguousarray(points).tobytes())
        else:
            f.write("".join(f"{x:.9g} {y:.9g} {z:.9g}\n" for x, y, z in points).encode("ascii"))


class IO:
    """utils/io.py:27-48 -- by file extension."""

    @classmethod
    def get(cls, file_path):
        ext = os.path.splitext(file_path)[1]
        if ext == ".npy":
            return np.load(file_path)              # allow_pickle stays False
        if ext == ".pcd":
            return read_pcd(file_path)
        if ext == ".txt":
            return np.loadtxt(file_path)
        if ext == ".h5":
            try:
                import h5py
            except ImportError as exc:             # not installed in this image
                raise RuntimeError("reading .h5 needs h5py") from exc
            with h5py.File(file_path, "r") as f:
                return f["data"][()]
        raise Exception("Unsupported file extension: %s" % ext)

    @classmethod
    def put(cls, file_path, file_content):
        ext = os.path.splitext(file_path)[1]
        if ext == ".pcd":
            return write_pcd(file_path, file_content)
        if ext == ".npy":
            return np.save(file_path, file_content)
        raise Exception("Unsupported file extension: %s" % ext)


# ------------------------------------------------------------------ transforms
class UpSamplePoints:
    """data_transforms.py:153-172."""

    def __init__(self, parameters):
        self.n_points = parameters["n_points"]

    def __call__(self, ptcloud):
        curr = ptcloud.shape[0]
        need = self.n_points - curr
        if need < 0:
            return ptcloud[np.random.permutation(self.n_points)]
        while curr <= need:                # whole copies first
            ptcloud = np.tile(ptcloud, (2, 1))
            need -= curr
            curr *= 2
        return np.concatenate((ptcloud, ptcloud[np.random.permutation(need)]))


class RandomSamplePoints:
    """data_transforms.py:175-187: a random subset, zero rows when short."""

    def __init__(self, parameters):
        self.n_points = parameters["n_points"]

    def __call__(self, ptcloud):
        ptcloud = ptcloud[np.random.permutation(ptcloud.shape[0])[:self.n_points]]
        if ptcloud.shape[0] < self.n_points:
            ptcloud = np.concatenate([ptcloud, np.zeros((self.n_points - ptcloud.shape[0], 3))])
        return ptcloud


def _mirror(axis):
    """transforms3d.zooms.zfdir2mat(-1, e_axis): I - 2 e e^T (reflection through
    the plane normal to the axis).  transforms3d (unpinned, not installed) is
    restated from its published definition, I + (factor - 1) d d^T for unit d."""
    m = np.eye(3)
    m[axis, axis] = -1.0
    return m


class RandomMirrorPoints:
    """data_transforms.py:228-245: rnd <= 0.25 mirror x and z; <= 0.5 x;
    <= 0.75 z; otherwise unchanged.  `rnd_value` is Compose's per-transform
    uniform draw (data_transforms.py:25-39)."""

    def __init__(self, parameters=None):
        pass

    def __call__(self, ptcloud, rnd_value):
        mx, mz = _mirror(0), _mirror(2)
        t = np.eye(3)
        if rnd_value <= 0.25:
            t = mz @ (mx @ t)
        elif rnd_value <= 0.5:
            t = mx @ t
        elif rnd_value <= 0.75:
            t = mz @ t
        ptcloud[:, :3] = np.dot(ptcloud[:, :3], t.T)
        return ptcloud


class ScalePoints:
    """data_transforms.py:213-226 (random scale 0.85-0.94 unless fixed)."""

    def __init__(self, parameters=None):
        self.scale = None

    def __call__(self, ptcloud, rnd_value):
        scale = self.scale if self.scale is not None else np.random.randint(85, 95) * 0.01
        return ptcloud * scale


class ToTensor:
    def __init__(self, parameters=None):
        pass

    def __call__(self, arr):
        return torch.from_numpy(np.ascontiguousarray(arr)).float()


class Compose:
    """data_transforms.py:14-42: each transform draws rnd_value = U(0, 1) once
    per sample and applies to the listed objects.  `transforms` are
    (instance, objects) pairs."""

    _RANDOM = (RandomMirrorPoints, ScalePoints)

    def __init__(self, transforms):
        self.transformers = list(transforms)

    def __call__(self, data):
        for transform, objects in self.transformers:
            rnd_value = np.random.uniform(0, 1)
            for k, v in data.items():
                if k in objects:
                    data[k] = transform(v, rnd_value) if isinstance(transform, self._RANDOM) else transform(v)
        return data


def pcn_train_transforms(n_input=2048, n_gt=16384):
    """core/train_pcn.py's train pipeline (data_loaders.py:136-151): partial
    up-sampled to 2048 points, both clouds mirrored together, to tensors."""
    return Compose([(UpSamplePoints({"n_points": n_input}), ["partial_cloud"]),
                    (RandomMirrorPoints(), ["partial_cloud", "gtcloud"]),
                    (ToTensor(), ["partial_cloud", "gtcloud"])])


# ------------------------------------------------------------------ ShapeNet-55
def pc_norm(pc):
    """data_loaders.py:221-227: centre on the centroid, scale the farthest point to radius 1."""
    pc = pc - np.mean(pc, axis=0)
    return pc / np.max(np.sqrt(np.sum(pc ** 2, axis=1)))


def collate(batch):
    """data_loaders.py:32-45: (taxonomy_ids, model_ids, {key: stacked tensor})."""
    tax, mids, data = [], [], {}
    for t, m, d in batch:
        tax.append(t)
        mids.append(m)
        for k, v in d.items():
            data.setdefault(k, []).append(v)
    return tax, mids, {k: torch.stack(v, 0) for k, v in data.items()}
