"""W3 phase profile (diagnostics): s_memtime stamps of wave 0 of 256 workgroups per phase of the second-order
kernel (w3_kernel.hpp), averaged. usage: python tools/w3_phases.py [theta|kept|plain]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(kind):
    import __graft_entry__
    __graft_entry__.build()
    from siren_amd import _lib
    from siren_amd.engine import SirenEngine
    from siren_amd.modules import FCBlock
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    d = 3 if kind == 'kept' else 2
    net = FCBlock(d, 1, 3, 256, outermost_linear=True, nonlinearity='sine')
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).to(dev)
    eng = SirenEngine(d, 256, 3, 1)
    ws = eng.pack(flat)
    n = 1 << 19
    x = torch.rand(n, d, device=dev) * 2 - 1
    v = torch.randn(n, d, device=dev)
    gy = torch.randn(n, 1, device=dev)
    stamps = torch.zeros(256, 16, dtype=torch.int64, device=dev)
    lib = _lib.load()

    def run():
        if kind == 'kept':
            _, _, kept = eng.forward_grad_store(ws, x)
            eng.second_order(ws, x, v, want_theta=True, gy=gy, kept=kept)
        else:
            eng.second_order(ws, x, v, want_theta=(kind == 'theta'))
    run()
    torch.cuda.synchronize()
    lib.siren_w3_phase_profile(ctypes.c_void_p(stamps.data_ptr()))
    run()
    torch.cuda.synchronize()
    lib.siren_w3_phase_profile(None)
    st = stamps.cpu().double()
    dt = (st[:, 1:] - st[:, :-1]).mean(0)
    names = ['layer0', 'fwd GEMM1', 'fwd epi1', 'fwd GEMM2', 'fwd epi2', 'fwd GEMM3', 'fwd epi3', 'seed',
             'rev GEMM3', 'rev epi3', 'rev GEMM2', 'rev epi2', 'rev GEMM1', 'rev epi1', 'gx']
    total = float(st[:, 15].sub(st[:, 0]).mean())
    print('kind', kind, 'total cycles per tile %.0f' % total)
    for nme, t in zip(names, dt.tolist()):
        print('  %-10s %9.0f  %5.1f%%' % (nme, t, 100 * t / total))


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'theta')
