"""HIP-event timing of the headline W1 launch, fp32 kernel vs the split-bf16 kernel, at N = 2^20 (5x256 d2 o1):
python tools/time_split.py [--n N] [--reps R]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    st = torch.cuda.current_stream()
    for _ in range(3):
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
    ap.add_argument('--n', type=int, default=1 << 20)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--d', type=int, default=2)
    a = ap.parse_args()
    from siren_amd.engine import SirenEngine
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(0)
    net = SingleBVPNet(in_features=a.d)
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).cuda()
    eng = SirenEngine(a.d, 256, 3, 1)
    ws, wsx = eng.pack(flat), eng.pack_split(flat)
    x = torch.rand(a.n, a.d, device='cuda') * 2 - 1
    F = 2 * (a.d * 256 + 3 * 256 * 256 + 256)
    out = {'n': a.n}
    for name, fn in (('fp32', lambda: eng.forward_grad(ws, x)), ('split_bf16x6', lambda: eng.forward_grad_split(wsx, x))):
        ms = timed(fn, a.reps)
        out[name] = {'ms': round(ms, 4), 'mcoords_s': round(a.n / ms / 1e3, 2),
                     'tflops_fp32_equiv': round(2 * F * a.n / ms / 1e9, 2),
                     'frac_fp32_peak': round(2 * F * a.n / ms / 1e9 / 157.3, 4)}
    for name, fn in (('fwd_fp32', lambda: eng.forward(ws, x)), ('fwd_split_bf16x6', lambda: eng.forward_split(wsx, x))):
        ms = timed(fn, a.reps)
        out[name] = {'ms': round(ms, 4), 'mcoords_s': round(a.n / ms / 1e3, 2),
                     'tflops_fp32_equiv': round(F * a.n / ms / 1e9, 2),
                     'frac_fp32_peak': round(F * a.n / ms / 1e9 / 157.3, 4)}
    out['pack_split_ms'] = round(timed(lambda: eng.pack_split(flat), 10), 4)
    y, g = eng.forward_grad(ws, x)
    ys, gs = eng.forward_grad_split(wsx, x)
    out['max_dy_vs_fp32'] = float((y - ys).abs().max())
    out['max_dg_vs_fp32'] = float((g - gs).abs().max())
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
