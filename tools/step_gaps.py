"""GPU idle time inside a training step: runs the bench's image-fit step (SingleBVPNet 5x256 d2, image_mse, torch
Adam; bench.py train_step_rate) and the hypernet leg's shape under the HIP event clock and prints wall ms per step; run
it under `rocprofv3 --kernel-trace` and pass the trace directory to report the kernels' busy time per step and the
idle gaps between them.   python tools/step_gaps.py [--n N] [--steps K] | python tools/step_gaps.py --trace DIR"""
import argparse
import csv
import glob
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(n, steps):
    import torch
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(0)
    dev = torch.device('cuda')
    model = SingleBVPNet(verbose=False, jet=False).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    x = torch.rand(1, n, 2, device=dev) * 2 - 1
    gt = torch.sin(5 * x[..., :1])

    def step():
        out = model({'coords': x})
        loss = ((out['model_out'] - gt) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    print('image_w2 n=%d: %.3f ms/step wall' % (n, (time.perf_counter() - t0) / steps * 1e3))


def trace(d, steps):
    f = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)[0]
    rows = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:50])
                   for r in csv.DictReader(open(f))), key=lambda t: t[0])
    rows = rows[-steps * 200:]
    busy = sum(e - s for s, e, _ in rows)
    span = rows[-1][1] - rows[0][0]
    gaps = sorted(((rows[i + 1][0] - rows[i][1], rows[i][2], rows[i + 1][2]) for i in range(len(rows) - 1)),
                  reverse=True)
    print('kernels %d, span %.3f ms, busy %.3f ms, idle %.3f ms' % (len(rows), span / 1e6, busy / 1e6,
                                                                    (span - busy) / 1e6))
    for g, a, b in gaps[:12]:
        print('  gap %8.1f us  %s -> %s' % (g / 1e3, a, b))


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=1 << 18)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--trace', default=None)
    a = ap.parse_args()
    if a.trace:
        trace(a.trace, a.steps)
    else:
        run(a.n, a.steps)
