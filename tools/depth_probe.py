"""W0 / W1 / W2 / W3 efficiency vs depth (hidden layers 1..5, hidden 256, d 2, o 1): separates per-layer costs
from code-size effects (the fully unrolled W1 body grows ~40 KB per hidden layer) and measures the 4..5-layer
stored split against the register-resident 1..3-layer kernels.
usage: python tools/depth_probe.py [--n N] [--layers 1,2,3,4,5]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=1 << 20)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--layers', default='1,2,3,4,5')
    a = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    from siren_amd.engine import SirenEngine
    dev = torch.device('cuda:0')
    x = torch.rand(a.n, 2, device=dev) * 2 - 1
    gy = torch.randn(a.n, 1, device=dev)
    v = torch.randn(a.n, 2, device=dev)
    for L in [int(t) for t in a.layers.split(',')]:
        eng = SirenEngine(2, 256, L, 1)
        torch.manual_seed(0)
        flat = (torch.rand(eng.param_count, device=dev) - 0.5) * 0.01
        ws = eng.pack(flat)
        F = 2 * (2 * 256 + L * 256 * 256 + 256)
        for name, fn, fl in (('W0', lambda: eng.forward(ws, x), F), ('W1', lambda: eng.forward_grad(ws, x), 2 * F),
                             ('W2', lambda: eng.backward_params(ws, x, gy), 3 * F),
                             ('W3th', lambda: eng.second_order(ws, x, v, want_theta=True), 6 * F)):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0.record()
                for _ in range(a.reps):
                    fn()
                s1.record()
                torch.cuda.synchronize()
                ts.append(s0.elapsed_time(s1) / a.reps)
            ms = min(ts)
            tf = fl * a.n / (ms * 1e-3) / 1e12
            print('L=%d %s %.3f ms  %.1f TFLOP/s  %.1f%% of 157.3' % (L, name, ms, tf, 100 * tf / 157.3), flush=True)


if __name__ == '__main__':
    main()
