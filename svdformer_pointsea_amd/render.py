"""Depth renderers on libpcops.so.

PCViews       <- models/model_utils.py:1179-1234 (SVDFormer; harmonic-mean depth splat)
PCViews_Real  <- models_PointSea/mv_utils_zs.py:136-195 (PointSea; voxel scatter-max,
                 7x7 max-pool, 3x3 Gaussian, max over depth, normalise)
The view rotation matrices are built exactly as the reference builds them
(euler2mat in torch float32, transposed); they are computed on the host CPU so
the product path does not depend on the device's sin/cos.
"""
import numpy as np
import torch

from . import _lib
from ._lib import call, lib, ptr, require_float, stream_of


def euler2mat(angle):
    """models/model_utils.py:952-1001 (also mv_utils_zs.py:46-94): [b,3] -> [b,3,3]."""
    x, y, z = angle[:, 0], angle[:, 1], angle[:, 2]
    b = angle.shape[0]
    cosz, sinz = torch.cos(z), torch.sin(z)
    zero = z.detach() * 0
    one = zero.detach() + 1
    zmat = torch.stack([cosz, -sinz, zero, sinz, cosz, zero, zero, zero, one], dim=1).reshape(b, 3, 3)
    cosy, siny = torch.cos(y), torch.sin(y)
    ymat = torch.stack([cosy, zero, siny, zero, one, zero, -siny, zero, cosy], dim=1).reshape(b, 3, 3)
    cosx, sinx = torch.cos(x), torch.sin(x)
    xmat = torch.stack([one, zero, zero, zero, cosx, -sinx, zero, sinx, cosx], dim=1).reshape(b, 3, 3)
    return xmat @ ymat @ zmat


class PCViews:
    """Three fixed views; get_img(points (B,N,3)) -> (B*3, R, R) depth images."""

    def __init__(self, TRANS, RESOLUTION):
        _views = np.asarray([
            [[0 * np.pi / 2, 0, np.pi / 2], [0, 0, TRANS]],
            [[1 * np.pi / 2, 0, np.pi / 2], [0, 0, TRANS]],
            [[0, -np.pi / 2, np.pi / 2], [0, 0, TRANS]]])
        self.num_views = 3
        angle = torch.tensor(_views[:, 0, :]).float()
        self.rot_mat = euler2mat(angle).transpose(1, 2).contiguous()
        self.translation = torch.tensor(_views[:, 1, :]).float().contiguous()
        self.resolution = RESOLUTION
        self._dev = {}

    def _consts(self, device):
        if device not in self._dev:
            self._dev[device] = (self.rot_mat.to(device), self.translation.to(device))
        return self._dev[device]

    def get_img(self, points):
        points = points.detach().contiguous()
        require_float(points, "points")
        B, N, _ = points.shape
        V, R = self.num_views, self.resolution
        rot, trans = self._consts(points.device)
        img = torch.empty(B * V, R, R, device=points.device)
        wsb = lib().pcops_points2depth_workspace_bytes(B, V, R, R)
        ws = _lib.Workspace.get(points.device, wsb)
        with torch.cuda.device(points.device):
            call("points2depth", lib().pcops_points2depth, ptr(points), ptr(rot), ptr(trans), B, N, V, R, R, ptr(img),
                 ptr(ws), wsb, stream_of(points))
        return img


# mv_utils_zs.py:9-14
params = {'maxpoolz': 1, 'maxpoolxy': 7, 'maxpoolpadz': 0, 'maxpoolpadxy': 3, 'convz': 1, 'convxy': 3,
          'convsigmaxy': 3, 'convsigmaz': 1, 'convpadz': 0, 'convpadxy': 1, 'imgbias': 0., 'depth_bias': 0.2,
          'obj_ratio': 0.8, 'bg_clr': 0.0, 'resolution': 224, 'depth': 8}


def get2DGaussianKernel(ksize, sigma=0):
    """mv_utils_zs.py:197-204."""
    center = ksize // 2
    xs = (np.arange(ksize, dtype=np.float32) - center)
    kernel1d = np.exp(-(xs ** 2) / (2 * sigma ** 2))
    kernel = kernel1d[..., None] @ kernel1d[None, ...]
    kernel = torch.from_numpy(kernel)
    return kernel / kernel.sum()


def get3DGaussianKernel(ksize, depth, sigma=2, zsigma=2):
    """mv_utils_zs.py:206-212."""
    kernel2d = get2DGaussianKernel(ksize, sigma)
    zs = (np.arange(depth, dtype=np.float32) - depth // 2)
    zkernel = np.exp(-(zs ** 2) / (2 * zsigma ** 2))
    kernel3d = np.repeat(kernel2d[None, :, :], depth, axis=0) * zkernel[:, None, None]
    return kernel3d / torch.sum(kernel3d)


class PCViews_Real:
    """get_img(points (B,N,3)) -> (B*3, 3, 224, 224) PointSea 'realistic' depth images."""

    def __init__(self, TRANS=-0.7):
        _views = np.asarray([
            [[0 * np.pi / 2, 0, np.pi / 2], [-0.5, -0.5, TRANS]],
            [[1 * np.pi / 2, 0, np.pi / 2], [-0.5, -0.5, TRANS]],
            [[0, -np.pi / 2, np.pi / 2], [-0.5, -0.5, TRANS]]])
        _views_bias = np.asarray([
            [[0, np.pi / 9, 0], [-0.5, 0, TRANS]],
            [[0, np.pi / 9, 0], [-0.5, 0, TRANS]],
            [[0, np.pi / 15, 0], [-0.5, 0, TRANS]]])
        self.num_views = _views.shape[0]
        self.rot_mat = euler2mat(torch.tensor(_views[:, 0, :]).float()).transpose(1, 2).contiguous()
        self.rot_mat2 = euler2mat(torch.tensor(_views_bias[:, 0, :]).float()).transpose(1, 2).contiguous()
        self.translation = torch.tensor(_views[:, 1, :]).float().contiguous()
        kern = get3DGaussianKernel(params['convxy'], params['convz'], sigma=params['convsigmaxy'],
                                   zsigma=params['convsigmaz'])
        self.kernel = torch.as_tensor(kern, dtype=torch.float32).reshape(3, 3).contiguous()
        self._dev = {}

    def _consts(self, device):
        if device not in self._dev:
            self._dev[device] = tuple(t.to(device) for t in (self.rot_mat, self.rot_mat2, self.translation,
                                                             self.kernel))
        return self._dev[device]

    def points2grid(self, points):
        """(B,N,3) -> voxel grid (B*3, 8, 224, 224), [img][z][x][y] (mv_utils_zs.py:97-133)."""
        points = points.detach().contiguous()
        require_float(points, "points")
        B, N, _ = points.shape
        R, D, V = params['resolution'], params['depth'], self.num_views
        rot, rot2, trans, _ = self._consts(points.device)
        grid = torch.empty(B * V, D, R, R, device=points.device)
        with torch.cuda.device(points.device):
            call("points2grid", lib().pcops_points2grid, ptr(points), ptr(rot), ptr(rot2), ptr(trans), B, N, V, R, D,
                 ptr(grid), stream_of(points))
        return grid

    def grid2image(self, grid):
        """Grid2Image (mv_utils_zs.py:16-43): (BV, D, R, R) -> (BV, 3, R, R)."""
        grid = grid.contiguous()
        BV, D, R, _ = grid.shape
        kern = self._consts(grid.device)[3]
        img = torch.empty(BV, 3, R, R, device=grid.device)
        wsb = lib().pcops_grid2image_workspace_bytes(BV, D, R)
        ws = _lib.Workspace.get(grid.device, wsb)
        with torch.cuda.device(grid.device):
            call("grid2image", lib().pcops_grid2image, ptr(grid), ptr(kern), BV, D, R, ptr(img), ptr(ws), wsb,
                 stream_of(grid))
        return img

    def get_img(self, points):
        return self.grid2image(self.points2grid(points))
