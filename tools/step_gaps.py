"""Where a drop-in training step's time goes: runs one bench training step (bench.py's loops: model -> loss_functions
-> backward -> torch Adam) for a path, prints wall ms per step; run it under `rocprofv3 --kernel-trace` and pass the
trace directory with --trace to list one steady-state step's kernels (duration, gap after) and the step's busy / idle.
  python tools/step_gaps.py --path image_w2|poisson|poisson_ref|sdf [--steps K]
  python tools/step_gaps.py --trace DIR --marker CatArray"""
import argparse
import csv
import glob
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(path, dev):
    import torch
    from siren_amd import dataio
    from siren_amd import loss_functions as LF
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(0)
    if path == 'image_w2':
        m = SingleBVPNet(verbose=False, jet=False).to(dev)
        x = torch.rand(1, 1 << 18, 2, device=dev) * 2 - 1
        gt = torch.sin(5 * x[..., :1])

        def loss_fn(out):
            return {'img': ((out['model_out'] - gt) ** 2).mean()}
    elif path in ('poisson', 'poisson_ref'):
        m = SingleBVPNet(verbose=False).to(dev)
        x = dataio.get_mgrid(512)[None].to(dev)
        lap_gt = torch.sin(4 * x[..., :1])
        if path == 'poisson':
            def loss_fn(out):
                return LF.laplace_mse(out, {'laplace': lap_gt})
        else:
            from bench import reference_laplace

            def loss_fn(out):
                return {'l': ((reference_laplace(out['model_out'], out['model_in']) - lap_gt) ** 2).mean()}
    elif path == 'sdf':
        m = SingleBVPNet(in_features=3, verbose=False).to(dev)
        inp, gt_sdf = dataio.sphere_sdf_batch(1 << 18, device=dev)
        x = inp['coords']

        def loss_fn(out):
            return LF.sdf(out, gt_sdf)
    else:
        raise ValueError(path)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)

    def step():
        out = m({'coords': x})
        total = sum(v.mean() for v in loss_fn(out).values())
        opt.zero_grad()
        total.backward()
        opt.step()
    return step, x.shape[1]


def run(path, steps):
    import torch
    step, n = build(path, torch.device('cuda'))
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    print('%s: %.3f ms/step wall, %.2f Mcoords/s' % (path, ms, n / ms / 1e3))


def trace(d, marker):
    f = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)[0]
    rows = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'])
                  for r in csv.DictReader(open(f)))
    idx = [i for i, r in enumerate(rows) if marker in r[2]]  # one marker kernel per step (the parameter cat)
    a, b = idx[-2], idx[-1]
    seg = rows[a:b + 1]
    span = (seg[-1][0] - seg[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in seg[:-1]) / 1e3
    print('one step: %d kernels, span %.1f us, busy %.1f us, idle %.1f us' % (len(seg) - 1, span, busy, span - busy))
    for i, (s, e, nm) in enumerate(seg[:-1]):
        print('%9.1f us  gap_after %7.1f  %s' % ((e - s) / 1e3, (seg[i + 1][0] - e) / 1e3, nm[:100]))


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--path', default='image_w2')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--trace', default=None)
    ap.add_argument('--marker', default='CatArray')
    a = ap.parse_args()
    if a.trace:
        trace(a.trace, a.marker)
    else:
        run(a.path, a.steps)
