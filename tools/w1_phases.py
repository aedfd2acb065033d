"""Per-phase cycle counts of the W1 kernel from siren_w1_phase_profile (s_memtime stamps per wave: tile start,
after each of the 6 GEMMs, tile end). usage: python tools/w1_phases.py [--n N]"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=1 << 20)
    ap.add_argument('--flags', type=int, default=0, help='cfg.reserved (SIREN_FLAG_ILV = 4)')
    a = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    from siren_amd import _lib
    from siren_amd.engine import SirenEngine, _ptr, _stream
    from bench import seed0_params
    dev = torch.device('cuda:0')
    eng = SirenEngine(2, 256, 3, 1, flags=a.flags)
    ws = eng.pack(seed0_params(dev))
    x = torch.rand(a.n, 2, device=dev) * 2 - 1
    y = torch.empty(a.n, 1, device=dev)
    gx = torch.empty(a.n, 2, device=dev)
    stamps = torch.zeros(256 * 4 * 4 * 8, dtype=torch.int64, device=dev)
    for _ in range(3):
        _lib.check(eng.lib.siren_w1_phase_profile(ctypes.byref(eng.cfg), _ptr(ws), _ptr(x), a.n, _ptr(y), _ptr(gx),
                                                  _ptr(stamps), _stream(dev)), 'profile')
    torch.cuda.synchronize()
    st = stamps.view(256, 4, 4, 8).cpu().numpy().astype(np.float64)
    ok = st[..., 7] > 0
    d = np.diff(st, axis=-1)  # 7 phases
    names = ['GEMM0 fwd (FIRST epi)', 'GEMM1 fwd (SINCOS)', 'GEMM2 fwd (SINCOS)', 'GEMM3 rev (SEED epi)',
             'GEMM4 rev (DELTA)', 'GEMM5 rev (DELTA)', 'tail (y, delta0, gx)']
    print('flags %d' % a.flags)
    print('s_memtime cycles per wave-tile phase (256 WGs x tiles 0..3 x 4 waves); ideal GEMM = 16 slices x 64 '
          'MFMA x 32 cyc = 32768')
    for t in range(4):
        sel = ok[:, t, :]
        row = ['%s %.0f' % (names[i], np.mean(d[:, t, :, i][sel])) for i in range(7)]
        tot = np.mean((st[:, t, :, 7] - st[:, t, :, 0])[sel])
        print('tile %d: total %.0f | %s' % (t, tot, ' | '.join(row)))
    # gaps between consecutive tiles (end of tile t -> start of tile t+1)
    gap = st[:, 1:, :, 0] - st[:, :-1, :, 7]
    print('inter-tile gap: %.0f cycles' % np.mean(gap[ok[:, 1:, :]]))
    # wave skew at GEMM ends
    sk = st.max(axis=2) - st.min(axis=2)
    print('wave skew per event (max-min over the 4 waves): %s' % np.round(np.mean(sk[ok[:, :, 0]], axis=0)))


if __name__ == '__main__':
    main()
