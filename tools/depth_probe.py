"""W0 / W1 kernel efficiency vs depth (hidden layers 1..3, hidden 256, d 2, o 1): separates per-layer costs from
code-size effects (the fully unrolled W1 body grows ~40 KB per hidden layer).
usage: python tools/depth_probe.py [--n N]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=1 << 20)
    ap.add_argument('--reps', type=int, default=10)
    a = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    from siren_amd.engine import SirenEngine
    dev = torch.device('cuda:0')
    x = torch.rand(a.n, 2, device=dev) * 2 - 1
    for L in (1, 2, 3):
        eng = SirenEngine(2, 256, L, 1)
        torch.manual_seed(0)
        flat = (torch.rand(eng.param_count, device=dev) - 0.5) * 0.01
        ws = eng.pack(flat)
        F = 2 * (2 * 256 + L * 256 * 256 + 256)
        for name, fn, fl in (('W0', lambda: eng.forward(ws, x), F), ('W1', lambda: eng.forward_grad(ws, x), 2 * F)):
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
