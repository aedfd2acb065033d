"""Times the engine entry points (HIP events on the launch stream) for one architecture:
python tools/time_paths.py [--hidden 512] [--layers 3] [--d 3] [--o 3] [--n 262144]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=5):
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
    ap.add_argument('--hidden', type=int, default=512)
    ap.add_argument('--layers', type=int, default=3)
    ap.add_argument('--d', type=int, default=3)
    ap.add_argument('--o', type=int, default=3)
    ap.add_argument('--n', type=int, default=1 << 18)
    a = ap.parse_args()
    from siren_amd.engine import SirenEngine
    from siren_amd.modules import FCBlock
    torch.manual_seed(0)
    net = FCBlock(a.d, a.o, a.layers, a.hidden, outermost_linear=True, nonlinearity='sine')
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).cuda()
    eng = SirenEngine(a.d, a.hidden, a.layers, a.o)
    ws = eng.pack(flat)
    x = torch.rand(a.n, a.d, device='cuda') * 2 - 1
    gy = torch.randn(a.n, a.o, device='cuda')
    H, L, d, o = a.hidden, a.layers, a.d, a.o
    F = 2 * (d * H + L * H * H + H * o)
    for name, fn, work in (('W0 forward', lambda: eng.forward(ws, x), F),
                           ('W1 forward+vjp_x', lambda: eng.forward_grad(ws, x, gy), 2 * F),
                           ('W2 backward (store+wgrad+small+reduce)', lambda: eng.backward_params(ws, x, gy), 3 * F)):
        report(name, timed(fn), work, a.n)
    if eng.stored_supported:
        # stored-forward split: the training forward keeps a_l / cos, the backward is reverse-only; a W2 unit is the
        # forward (W0 role) + the backward, so compare W0 + W2-backward above with this pair
        state = {}

        def fwd_store():
            state['y'], state['tws'] = eng.forward_store(ws, x)
        fwd_store()
        t_fs = timed(fwd_store)
        t_bs = timed(lambda: eng.backward_stored(ws, x, gy, state['tws']))
        report('W2 split: forward_store', t_fs, F, a.n)
        report('W2 split: backward_stored (rev+wgrad+...)', t_bs, 2 * F, a.n)
        report('W2 split: forward_store + backward_stored', t_fs + t_bs, 3 * F, a.n)
        t_w0, t_w2 = timed(lambda: eng.forward(ws, x)), timed(lambda: eng.backward_params(ws, x, gy))
        report('W2 recompute: forward + backward_params', t_w0 + t_w2, 3 * F, a.n)
    if eng.laplace_supported:
        # W4 algorithmic unit: (1 + 2d) F; the jet kernel executes 4F (4 MFMA columns/coord)
        report('W4 y+grad+Laplacian (jet, 1 launch)', timed(lambda: eng.forward_laplace(ws, x, True, True)),
               (1 + 2 * d) * F, a.n)
        # laplace_mse training kernels (W4s unit 3 (1 + 2d) F): W4 + W4s recompute vs the split pair
        gl = torch.randn(a.n, 1, device='cuda')
        t_r = timed(lambda: eng.forward_laplace(ws, x)) + timed(lambda: eng.laplace_backward(ws, x, gl))
        jst = {}

        def lfs():
            jst['lap'], jst['tws'] = eng.forward_laplace_store(ws, x)
        lfs()
        t_s = timed(lfs) + timed(lambda: eng.laplace_backward_stored(ws, x, gl, jst['tws']))
        report('W4s train kernels, recompute (W4 + W4s)', t_r, 3 * (1 + 2 * d) * F, a.n)
        report('W4s train kernels, split (store + reverse)', t_s, 3 * (1 + 2 * d) * F, a.n)
    if eng.second_order_supported:
        v = torch.randn(a.n, a.d, device='cuda')
        for name, fn, work in (('W3 H v (x only)', lambda: eng.second_order(ws, x, v, want_theta=False), 4 * F),
                               ('W3 H v + theta-grad', lambda: eng.second_order(ws, x, v, want_theta=True), 6 * F)):
            report(name, timed(fn), work, a.n)
        if eng.stored_supported and a.o == 1:
            # sdf step kernels: jet forward (y, J) + seeded W3 with theta-grads, recompute vs stored forward
            gy1 = torch.randn(a.n, 1, device='cuda')
            st = {}

            def fwd_keep():
                st['y'], st['J'], st['k'] = eng.forward_grad_store(ws, x)
            fwd_keep()
            t_fk = timed(fwd_keep)
            t_bk = timed(lambda: eng.second_order(ws, x, v, want_theta=True, gy=gy1, kept=st['k']))
            t_fr = timed(lambda: eng.forward_grad(ws, x))
            t_br = timed(lambda: eng.second_order(ws, x, v, want_theta=True, gy=gy1))
            report('sdf kernels, stored: fwd_grad_store', t_fk, 2 * F, a.n)
            report('sdf kernels, stored: W3 kept + theta', t_bk, 6 * F, a.n)
            report('sdf kernels, stored: total (8F)', t_fk + t_bk, 8 * F, a.n)
            report('sdf kernels, recompute: total (8F)', t_fr + t_br, 8 * F, a.n)


def report(name, ms, work, n):
    print('%-42s %8.3f ms  %8.2f Mcoords/s  %6.1f TFLOP/s (%.1f%% of 157.3)'
          % (name, ms, n / ms / 1e3, work * n / ms / 1e9, work * n / ms / 1e9 / 157.3 * 100), flush=True)


if __name__ == '__main__':
    main()
