"""Grouped (one launch over the batch) vs per-element launches for batched hypernetwork weights:
python tools/time_batched.py [--B 32] [--n 4096]. HIP events on the launch stream; W0 = forward, W1 = fwd + grad,
5x256 d2 o1 hypo-network (the neural-process setting: meta-batch of 64x64 images)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=10):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--B', type=int, default=32)
    ap.add_argument('--n', type=int, default=4096)
    a = ap.parse_args()
    from siren_amd.engine import SirenEngine
    eng = SirenEngine(2, 256, 3, 1)
    P = eng.param_count
    flat = torch.randn(a.B, P, device='cuda') * 0.01
    x = torch.rand(a.B, a.n, 2, device='cuda') * 2 - 1
    wsb = eng.pack_batched(flat)
    F = 394752
    gy = torch.randn(a.B, a.n, 1, device='cuda')
    for name, grouped, single, flop in (
            ('W2 backward', lambda: eng.backward_params_batched(wsb, x, gy),
             lambda b: eng.backward_params(wsb[b], x[b], gy[b]), 3 * F),  # store (fwd + rev) + wgrad
            ('W0 forward', lambda: eng.forward_batched(wsb, x), lambda b: eng.forward(wsb[b], x[b]), F),
            ('W1 fwd+grad', lambda: eng.forward_grad_batched(wsb, x), lambda b: eng.forward_grad(wsb[b], x[b]), 2 * F)):
        tg = timed(grouped)
        tl = timed(lambda: [single(b) for b in range(a.B)])
        coords = a.B * a.n
        print('%-12s B=%d n=%d: grouped %.3f ms (%.1f Mcoords/s, %.1f%% of fp32 peak) | per-element %.3f ms (%.1f '
              'Mcoords/s) | %.2fx' % (name, a.B, a.n, tg, coords / tg / 1e3, coords * flop / tg / 1e9 / 157.3 * 100,
                                      tl, coords / tl / 1e3, tl / tg), flush=True)


if __name__ == '__main__':
    main()
