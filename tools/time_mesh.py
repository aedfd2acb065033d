"""Timing of sdf_meshing on the device: the dense decoder evaluation of create_mesh on the
fused W0 kernel (5x256 d3 SIREN, N^3 voxels) and the device marching cubes (marching.hip) on its volume. One JSON
line per N. usage: python tools/time_mesh.py [--precision fp32|bf16x6] [N ...]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(Ns, precision='fp32'):
    import __graft_entry__
    __graft_entry__.build()
    from siren_amd import sdf_meshing as M
    from siren_amd.modules import SingleBVPNet
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    m = SingleBVPNet(in_features=3, verbose=False, precision=precision).to(dev)
    dec = lambda c: m({'coords': c})['model_out']  # noqa: E731
    dec.parameters = m.parameters
    for N in Ns:
        sdf = M.evaluate_sdf_grid(dec, N, device=dev, out_device=dev)
        level = float(sdf.median())
        M.marching_cubes(sdf, level)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sdf = M.evaluate_sdf_grid(dec, N, device=dev, out_device=dev)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            v, f = M.marching_cubes(sdf, level, (2. / (N - 1),) * 3)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        mc_ms = (t2 - t1) / reps * 1e3
        print(json.dumps({'N': N, 'precision': precision, 'voxels': N ** 3, 'eval_ms': round((t1 - t0) * 1e3, 2),
                          'eval_mcoords_s': round(N ** 3 / (t1 - t0) / 1e6, 1), 'mc_ms': round(mc_ms, 3),
                          'mc_gvox_s': round(N ** 3 / mc_ms / 1e6, 2), 'verts': int(v.shape[0]),
                          'faces': int(f.shape[0])}), flush=True)


if __name__ == '__main__':
    args = sys.argv[1:]
    prec = 'fp32'
    if len(args) >= 2 and args[0] == '--precision':
        prec, args = args[1], args[2:]
    main([int(a) for a in args] or [256, 512], prec)
