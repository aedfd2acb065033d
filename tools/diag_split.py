"""Locates split-bf16 W1 mismatches against the fp32 kernel by coordinate tile / wave / lane."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from siren_amd.engine import SirenEngine
from siren_amd.modules import SingleBVPNet

torch.manual_seed(0)
net = SingleBVPNet(in_features=2)
flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).cuda()
eng = SirenEngine(2, 256, 3, 1)
ws, wsx = eng.pack(flat), eng.pack_split(flat)
for n in (16384, 16384 + 64, 32768, 1 << 20):
    x = torch.rand(n, 2, device='cuda') * 2 - 1
    y, g = eng.forward(ws, x), None
    y32, g32 = eng.forward_grad(ws, x)
    ys, gs = eng.forward_grad_split(wsx, x)
    err = (gs - g32).abs().max(dim=1).values + (ys - y32).abs()[:, 0]
    bad = (err > 1e-4).nonzero()[:, 0]
    tiles = (bad // 64)
    print('n', n, 'bad', bad.numel(), 'max', float(err.max()))
    if bad.numel():
        t = tiles.unique()
        print('  tiles', t[:20].tolist(), '... count', t.numel(), ' tile//256 (round)', (t // 256).unique()[:10].tolist())
        w = ((bad % 64) // 16).unique().tolist()
        print('  waves', w, ' lanes c', (bad % 16).unique().tolist()[:16])
        print('  first bad coords', bad[:10].tolist())
