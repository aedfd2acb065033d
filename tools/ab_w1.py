"""In-process A/B of W1 kernel variants (interleaved rounds, one process: cdna guide §5.4 rule 24).
usage: python tools/ab_w1.py [--n N] [--rounds R] [--variants 0,1,2]   (variant = cfg.reserved flags)"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=1 << 20)
    ap.add_argument('--rounds', type=int, default=8)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--variants', default='0,1')
    ap.add_argument('--fwd', action='store_true', help='time siren_forward (W0) instead of W1')
    a = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    from siren_amd.engine import SirenEngine
    from oracle import siren_oracle as O
    from bench import seed0_params, W1_FLOP
    dev = torch.device('cuda:0')
    flat = seed0_params(dev)
    x = torch.rand(a.n, 2, device=dev) * 2 - 1
    variants = [int(v) for v in a.variants.split(',')]
    engs = {v: SirenEngine(2, 256, 3, 1, flags=v) for v in variants}
    ws = engs[variants[0]].pack(flat)
    outs = {}
    for v, e in engs.items():
        y, g = e.forward_grad(ws, x)
        outs[v] = (y, g)
    torch.cuda.synchronize()
    layers = O.unflatten(flat.cpu().numpy().astype(np.float64), 2, 256, 3, 1)
    idx = torch.randperm(a.n)[:2048].to(dev)
    ry, rg = O.forward_grad(x[idx].cpu().numpy(), layers)
    for v, (y, g) in outs.items():
        print('variant %d: max|dy| %.2e max|dg|/max|g| %.2e' % (v, np.max(np.abs(y[idx].cpu().numpy() - ry)),
              np.max(np.abs(g[idx].cpu().numpy() - rg)) / np.max(np.abs(rg))), flush=True)
    times = {v: [] for v in variants}
    for r in range(a.rounds):
        for v, e in engs.items():
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(a.reps):
                if a.fwd:
                    e.forward(ws, x, out=outs[v][0])
                else:
                    e.forward_grad(ws, x, out_y=outs[v][0], out_gx=outs[v][1])
            s1.record()
            torch.cuda.synchronize()
            times[v].append(s0.elapsed_time(s1) / a.reps)
    flop = W1_FLOP // 2 if a.fwd else W1_FLOP
    for v, (y, g) in outs.items():
        if a.fwd:
            y0 = e.forward(ws, x)
            print('variant %d forward: max|dy| %.2e' % (v, np.max(np.abs(engs[v].forward(ws, x)[idx].cpu().numpy() - ry))))
    for v, t in times.items():
        t = np.array(t)
        tf = flop * a.n / (np.median(t) * 1e-3) / 1e12
        print('variant %d: median %.3f ms  min %.3f ms  -> %.1f TFLOP/s (%.1f%% of 157.3)  %.1f Mcoords/s'
              % (v, np.median(t), t.min(), tf, tf / 157.3 * 100, a.n / np.median(t) / 1e3), flush=True)


if __name__ == '__main__':
    main()
