"""Per-phase cycle stamps of qf_rev_kernel (probe library built with -DQF_PROF: tools/variant_build.sh qfprof
"-DQF_PROF" tu_hess; SIREN_AMD_LIB=tools/probe/lib_qfprof.so): the kept Hessian backward at the poisson_ref size,
wave 0 of the first 256 workgroups, median cycles of the seed epilogue, each reverse GEMM and each epilogue."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from siren_amd.engine import SirenEngine, _ptr, _stream  # noqa: E402

n, L = 512 * 512, 3
eng = SirenEngine(2, 256, L, 1)
flat = (torch.rand(eng.param_count, device='cuda') * 2 - 1) * 0.05
ws = eng.pack(flat)
x = torch.rand(n, 2, device='cuda') * 2 - 1
G = torch.randn(n, 2, 2, device='cuda') / n
hm, kept = eng.hessian(ws, x, None, keep=True)
cnt = ctypes.c_int64()
eng.lib.siren_hessian_backward_ws_floats(ctypes.byref(eng.cfg), n, ctypes.byref(cnt))
tws = torch.empty(cnt.value, device='cuda')
gx = torch.zeros(max(n * 2, 256 * 32), device='cuda')
gp = torch.empty(eng.param_count, device='cuda')
for rep in range(3):
    eng.lib.siren_hessian_backward_kept(ctypes.byref(eng.cfg), _ptr(ws), _ptr(x), n, _ptr(G), None, _ptr(kept),
                                        _ptr(tws), _ptr(gx), None, None, _stream(x.device))
torch.cuda.synchronize()
st = gx[:256 * 32].view(torch.int64).view(256, 16).cpu().numpy().astype(np.int64)
ev = 2 + 2 * L
d = np.diff(st[:, :ev], axis=1)
names = ['seed epilogue'] + sum([['GEMM %d' % i, 'epilogue %d' % i] for i in range(L)], [])
for i, nm in enumerate(names):
    print('%-14s median %8.0f  p10 %8.0f  p90 %8.0f  (s_memtime ticks)' % (nm, np.median(d[:, i]),
          np.percentile(d[:, i], 10), np.percentile(d[:, i], 90)))
print('total          median %8.0f' % np.median(st[:, ev - 1] - st[:, 0]))
