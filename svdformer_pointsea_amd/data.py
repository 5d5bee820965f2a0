"""On-device data preparation of the ShapeNet-55 train loop.

seprate_point_cloud   utils/helpers.py:62-123 (online cropping: the points
                      nearest a random unit-sphere centre are cut away, the
                      rest is FPS-subsampled to 2048), called inside the
                      step by core/train_55.py:150.

The reference loops over the batch and issues two FPS launches per sample
on ragged clouds (N - num_crop and num_crop points).  Here the whole batch
goes through two batched FPS launches: every sample's kept (or cropped)
points are packed to the front of a (B, N_max, 3) buffer and the tail is
zero-filled.  That is exact, not an approximation: the FPS kernel never
selects a point with |p|^2 <= 1e-3 and never lets one update the running
distances (sampling_gpu.cu:100-101), the surviving points keep their
indices, and the block size (hence the tie rule) is 512 for every N >= 512,
so the selected indices are those of the per-sample ragged call.
"""
import os
import random

import torch
import torch.nn.functional as F

from ._lib import fork
from .model_utils import fps_subsample, fps_subsample_counts

# PCOPS_FPS_COUNTS=0: the crop FPS sweeps the whole zero-padded width (A/B runs)
_FPS_COUNTS = os.environ.get("PCOPS_FPS_COUNTS", "1") != "0"
# PCOPS_CROP_FUSED=0: the crop's order and packing by torch.argsort + _pack (~30 launches) instead of
# pcops_crop_pack (one launch) -- A/B runs and the bitwise test
_CROP_FUSED = os.environ.get("PCOPS_CROP_FUSED", "1") != "0"


def _pack(points, order, start, count, n_max):
    """rows order[b, start[b] : start[b] + count[b]] of points[b], packed to the
    front of a (B, n_max, 3) buffer with a zero tail."""
    B, N, _ = points.shape
    j = torch.arange(n_max, device=points.device).unsqueeze(0)
    src = (start.unsqueeze(1) + j).clamp_(max=N - 1)
    keep = j < count.unsqueeze(1)
    idx = torch.gather(order, 1, src)
    out = torch.gather(points, 1, idx.unsqueeze(-1).expand(B, n_max, 3))
    return out * keep.unsqueeze(-1).to(out.dtype)


def _crop_pack(dist, xyz, start, count, n_max):
    """_pack(xyz, argsort(dist), start, count, n_max) in one launch (pcops_crop_pack: the sort is stable,
    as the segmented radix sort torch.argsort runs) -> (packed (B, n_max, 3), counts (B,) int32, where
    count None means N - start)."""
    from ._lib import call, lib, ptr, stream_of

    B, N, _ = xyz.shape
    dist, xyz = dist.contiguous(), xyz.contiguous()
    start = start.to(torch.int64).contiguous()
    count = count.to(torch.int64).contiguous() if count is not None else None
    out = torch.empty(B, n_max, 3, device=xyz.device, dtype=xyz.dtype)
    counts = torch.empty(B, dtype=torch.int32, device=xyz.device)
    with torch.cuda.device(xyz.device):
        call("crop_pack", lib().pcops_crop_pack, ptr(dist), ptr(xyz), ptr(start), ptr(count), B, N, n_max, ptr(out),
             ptr(counts), stream_of(xyz))
    return out, counts


def seprate_point_cloud(xyz, num_points, crop, fixed_points=None, padding_zeros=False, generator=None,
                        want_crop=True):
    """utils/helpers.py:62-123 -> (input_data, crop_data).

    crop: int, or [lo, hi] for a per-sample random crop size (then both parts
    are FPS-subsampled to 2048, as the reference does).  fixed_points: None
    (random unit centre per sample), one (3,) point or a list to sample from.
    `generator` (optional, a torch.Generator on xyz's device) replaces the
    reference's global `random` / `torch.randn` draws for reproducible runs.
    want_crop=False returns (input_data, None) without the crop part's FPS: the
    train loop discards it (core/train_55.py:150 `partial, _ = ...`), FPS draws
    no random numbers, so input_data is unchanged."""
    B, n, c = xyz.shape
    assert n == num_points
    assert c == 3
    if crop == num_points:
        return xyz, None
    dev = xyz.device
    if isinstance(crop, list):
        if generator is None:
            num_crop = torch.tensor([random.randint(crop[0], crop[1]) for _ in range(B)], device=dev)
        else:
            num_crop = torch.randint(crop[0], crop[1] + 1, (B,), device=dev, generator=generator)
    else:
        num_crop = torch.full((B,), int(crop), device=dev)
    if fixed_points is None:
        if generator is None:
            center = F.normalize(torch.randn(B, 1, 3), p=2, dim=-1).to(dev)
        else:
            center = F.normalize(torch.randn(B, 1, 3, device=dev, generator=generator), p=2, dim=-1)
    else:
        pts = fixed_points if isinstance(fixed_points, list) else [fixed_points]
        center = torch.stack([torch.as_tensor(random.sample(pts, 1)[0], dtype=xyz.dtype).reshape(1, 3)
                              for _ in range(B)]).to(dev)
    dist = torch.norm(center - xyz, p=2, dim=-1)           # (B, n)
    fused = (_CROP_FUSED and isinstance(crop, list) and not padding_zeros and xyz.is_cuda
             and xyz.dtype == torch.float32 and n <= 16384)
    order = None if fused else torch.argsort(dist, dim=-1, descending=False)
    if padding_zeros:
        keep = torch.arange(n, device=dev).unsqueeze(0) >= num_crop.unsqueeze(1)
        mask = torch.zeros(B, n, dtype=torch.bool, device=dev).scatter_(1, order, keep)
        input_data = xyz * mask.unsqueeze(-1).to(xyz.dtype)
    if isinstance(crop, list):
        hi = int(crop[1])
        in_counts = None
        if fused:
            input_data, in_counts = _crop_pack(dist, xyz, num_crop, None, n - int(crop[0]))
        elif not padding_zeros:
            input_data = _pack(xyz, order, num_crop, n - num_crop, n - int(crop[0]))
        # the packed clouds are zero-padded past their valid rows; on the GPU the FPS sweep stops
        # at each cloud's count (the same points: the reference skips the zero rows)
        def fps(cloud, count, count32=None):
            if padding_zeros or not cloud.is_cuda or not _FPS_COUNTS:
                return fps_subsample(cloud.contiguous(), 2048)
            return fps_subsample_counts(cloud.contiguous(), count.to(torch.int32) if count32 is None else count32, 2048)

        if not want_crop:
            return fps(input_data, n - num_crop, in_counts), None
        cr_counts = None
        if fused:
            crop_data, cr_counts = _crop_pack(dist, xyz, torch.zeros_like(num_crop), num_crop, hi)
        else:
            crop_data = _pack(xyz, order, torch.zeros_like(num_crop), num_crop, hi)
        # the two FPS launches (B workgroups each) run side by side
        crop_data = crop_data.contiguous()
        with fork(dev, inputs=(crop_data, num_crop) + ((cr_counts,) if cr_counts is not None else ())) as br:
            crop_out = fps(crop_data, num_crop, cr_counts)
        input_out = fps(input_data, n - num_crop, in_counts)
        return input_out, br.join(crop_out)
    k = int(crop)
    if not padding_zeros:
        input_data = torch.gather(xyz, 1, order[:, k:].unsqueeze(-1).expand(B, n - k, 3))
    if not want_crop:
        return input_data.contiguous(), None
    crop_data = torch.gather(xyz, 1, order[:, :k].unsqueeze(-1).expand(B, k, 3))
    return input_data.contiguous(), crop_data.contiguous()
