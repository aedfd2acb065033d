"""Kernel-only timing of the per-step kernels under rocprofv3 (sample_sdf_kernel at k = 2^18, sumsq + adam over
the 5x256 d3 bucket): python tools/step_kernels.py, run as `rocprofv3 --kernel-trace --stats -- python3 ...`."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from siren_amd.dataio import PointCloud
    from siren_amd.optim import FusedAdam
    dev = torch.device('cuda')
    d = np.random.default_rng(0).normal(size=(1 << 20, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pcd = PointCloud(points=np.concatenate([d * 0.5, d], 1), on_surface_points=1 << 18, device=dev)
    params = [torch.nn.Parameter(torch.randn(198658, device=dev) * 0.01)]
    opt = FusedAdam(params, lr=1e-4, max_norm=1.)
    params[0].grad.normal_()
    for i in range(50):
        pcd.sample(i)
        opt.step()
    torch.cuda.synchronize()
    print('done')


if __name__ == '__main__':
    main()
