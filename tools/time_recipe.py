"""Times the module-level Poisson training step (BASELINE config 5) through the reference's own op sequence —
laplace = divergence(gradient()) (diff_operators.py:27-43) inside laplace_mse (loss_functions.py:104-109), then
backward and Adam — and optionally the fused siren_amd laplace(); run under rocprofv3 --kernel-trace --stats to see
the kernels of one step.

python tools/time_recipe.py [--fused] [--steps K]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--fused', action='store_true')
    ap.add_argument('--steps', type=int, default=5)
    a = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    import bench
    from siren_amd.modules import SingleBVPNet
    from siren_amd import dataio, loss_functions as LF
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    m = SingleBVPNet(verbose=False).to(dev)
    grid = dataio.get_mgrid(512)[None].to(dev)
    gt = torch.sin(4 * grid[..., :1])
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)

    def step():
        out = m({'coords': grid})
        if a.fused:
            loss = LF.laplace_mse(out, {'laplace': gt})['laplace_loss']
        else:
            loss = ((bench.reference_laplace(out['model_out'], out['model_in']) - gt) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    print('%s: %.3f ms/step, %.3f Mcoords/s' % ('fused' if a.fused else 'reference recipe', ms,
                                                grid.shape[1] / ms / 1e3), flush=True)


if __name__ == '__main__':
    main()
