"""Coordinate inputs of the hot path: get_mgrid (dataio.py:20-40) and the synthetic stand-ins for the
reference's datasets. Data loading proper (images, point clouds, video) is out of scope."""
import math

import numpy as np
import torch


def get_mgrid(sidelen, dim=2):
    """Flattened ij-ordered grid in [-1, 1]^dim, float32, shape (prod(sidelen), dim)."""
    if isinstance(sidelen, int):
        sidelen = dim * (sidelen,)
    if dim not in (2, 3):
        raise NotImplementedError('Not implemented for dim=%d' % dim)
    grids = np.mgrid[tuple(slice(0, s) for s in sidelen)]
    pc = np.stack(grids, axis=-1)[None, ...].astype(np.float32)
    for i in range(dim):
        den = max(sidelen[i] - 1, 1) if (dim == 3 and i == 0) else (sidelen[i] - 1)
        pc[..., i] = pc[..., i] / den
    pc -= 0.5
    pc *= 2.
    return torch.Tensor(pc).view(-1, dim)


def synthetic_image(coords):
    """0.6 (sin 8x cos 5y + 0.5 sign(sin 20xy)): the closed-form stand-in for the camera image."""
    x, y = coords[..., 0:1], coords[..., 1:2]
    return 0.6 * (torch.sin(8 * x) * torch.cos(5 * y) + 0.5 * torch.sign(torch.sin(20 * x * y)))


def synthetic_video(coords):
    """RGB in [0,1] on (t, x, y) coordinates: the stand-in for the 64x512x512 video volume."""
    return 0.5 + 0.5 * torch.sin(3 * coords + torch.tensor([0., 1., 2.], device=coords.device, dtype=coords.dtype))


def sphere_sdf_batch(on_surface_points, generator=None, device='cpu', radius=0.5):
    """PointCloud-shaped batch (dataio.py:420-442) for a sphere: on-surface points with unit normals and sdf 0,
    then the same number of uniform off-surface points with sdf -1 and normals -1."""
    n = on_surface_points
    on = torch.randn(n, 3, generator=generator, dtype=torch.float64)
    nrm = on / on.norm(dim=-1, keepdim=True)
    off = torch.rand(n, 3, generator=generator, dtype=torch.float64) * 2 - 1
    coords = torch.cat([nrm * radius, off], 0).float()
    normals = torch.cat([nrm, -torch.ones(n, 3, dtype=torch.float64)], 0).float()
    sdf = torch.cat([torch.zeros(n, 1), -torch.ones(n, 1)], 0)
    return ({'coords': coords[None].to(device)},
            {'sdf': sdf[None].to(device), 'normals': normals[None].to(device)})


def psnr(pred, gt):
    """PSNR as utils.py:578-587 / 316: [-1,1] -> [0,1], clip the prediction, data_range 1."""
    p = torch.clamp(pred / 2. + 0.5, 0., 1.).double()
    t = (gt / 2. + 0.5).double()
    mse = torch.mean((p - t) ** 2).item()
    return 10. * math.log10(1. / mse) if mse > 0 else float('inf')
