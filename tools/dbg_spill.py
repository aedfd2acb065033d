"""Debug: compare the W3 spill buffers (zdot per layer) of w3i and the serial w3 kernel."""
import sys, os, ctypes
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, 'tests'))
import numpy as np, torch
import __graft_entry__
__graft_entry__.build()
from siren_amd.engine import SirenEngine, _ptr, _stream
from oracle import siren_oracle as O
from test_gpu_parity import random_layers, to_dev
cuda = torch.device('cuda:0')
L, d, o, n = 2, 2, 1, 64
res = {}
for fl in (0, 4):
    e = SirenEngine(d, 256, L, o, flags=fl)
    ws = e.pack(to_dev(O.flatten(random_layers(d, L, o, seed=40)), cuda))
    rng = np.random.default_rng(L + n)
    x = to_dev(rng.uniform(-1, 1, (n, d)), cuda)
    v = to_dev(rng.normal(size=(n, d)), cuda)
    cnt = ctypes.c_int64()
    e.lib.siren_second_order_ws_floats(ctypes.byref(e.cfg), n, 0, ctypes.byref(cnt))
    tws = torch.full((cnt.value,), float('nan'), device=cuda)
    gx = torch.empty(n, d, device=cuda)
    rc = e.lib.siren_second_order_ex(ctypes.byref(e.cfg), _ptr(ws), _ptr(x), n, _ptr(v), None, None, _ptr(tws), _ptr(gx),
                                     None, None, _stream(cuda))
    torch.cuda.synchronize()
    sp = tws[:n // 16 * (L + 1) * 3 * 16 * 256].view(n // 16, L + 1, 3, 16, 64, 4).cpu().numpy()
    res[fl] = (sp, gx.cpu().numpy())
si, ss = res[0][0], res[4][0]
for l in range(L):
    dz = np.abs(si[:, l, 1] - ss[:, l, 1])  # zdot: (tile, block, lane, r)
    lanes = sorted(set(np.nonzero(dz.max(axis=(0, 1, 3)) > 0)[0].tolist()))
    print('layer %d zdot max diff %.3g, lanes differing %s' % (l, dz.max(), lanes))
    # z (w3i q=0) vs serial: serial q=0 holds cos -> compare cos(w z)
    w = 30.
    cz = np.cos(w * si[:, l, 0]); dc = np.abs(cz - ss[:, l, 0])
    lanes = sorted(set(np.nonzero(dc.max(axis=(0, 1, 3)) > 1e-3)[0].tolist()))
    print('layer %d cos(w z) vs serial cos max diff %.3g, lanes differing %s' % (l, dc.max(), lanes))
dg = np.abs(res[0][1] - res[4][1]).max(axis=1)
print('gx rows differing', np.nonzero(dg > 0)[0].tolist())
