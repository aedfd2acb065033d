"""Times full training steps through the drop-in API (model -> loss_functions -> backward -> Adam) per loss:
python tools/time_train.py [--n 262144] [--steps 10]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=1 << 18)
    ap.add_argument('--steps', type=int, default=10)
    a = ap.parse_args()
    from siren_amd.modules import SingleBVPNet
    from siren_amd import loss_functions as LF
    dev = torch.device('cuda')
    for loss, d in (('image_mse', 2), ('gradients_mse', 2), ('laplace_mse', 2), ('sdf', 3)):
        torch.manual_seed(0)
        m = SingleBVPNet(in_features=d, verbose=False).to(dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-4)
        x = torch.rand(1, a.n, d, device=dev) * 2 - 1
        gt = {'img': torch.sin(5 * x[..., :1]), 'gradients': torch.cos(3 * x[..., :2]),
              'laplace': torch.sin(4 * x[..., :1]), 'sdf': x.norm(dim=-1, keepdim=True) - 0.5,
              'normals': x / x.norm(dim=-1, keepdim=True)}

        def step():
            out = m({'coords': x})
            if loss == 'image_mse':
                terms = LF.image_mse(None, out, gt)
            else:
                terms = getattr(LF, loss)(out, gt)
            total = sum(v.mean() for v in terms.values())
            opt.zero_grad()
            total.backward()
            opt.step()
        step()
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        print('%-14s d=%d N=%d: %8.3f ms/step  %8.2f Mcoords/s' % (loss, d, a.n, ms, a.n / ms / 1e3), flush=True)


if __name__ == '__main__':
    main()
