"""Debug: grouped W3i vs serial vs per-element single calls (where do they differ?)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
import numpy as np, torch
import __graft_entry__
__graft_entry__.build()
from siren_amd.engine import SirenEngine
from oracle import siren_oracle as O
from test_gpu_parity import random_layers, to_dev
cuda = torch.device('cuda:0')
for (L, B, n) in [(2, 2, 64), (3, 2, 128), (2, 3, 64)]:
    d, o = 2, 1
    ei, es = SirenEngine(d, 256, L, o), SirenEngine(d, 256, L, o, flags=4)
    flats = torch.stack([to_dev(O.flatten(random_layers(d, L, o, seed=40 + b)), cuda) for b in range(B)])
    wi, wsr = ei.pack_batched(flats, full=True), es.pack_batched(flats, full=True)
    rng = np.random.default_rng(L + n)
    x = to_dev(rng.uniform(-1, 1, (B, n, d)), cuda)
    v = to_dev(rng.normal(size=(B, n, d)), cuda)
    gi, _ = ei.second_order_batched(wi, x, v, want_theta=False)
    gs, _ = es.second_order_batched(wsr, x, v, want_theta=False)
    for b in range(B):
        g1, _ = ei.second_order(wi[b], x[b], v[b], want_theta=False)
        g2, _ = es.second_order(wsr[b], x[b], v[b], want_theta=False)
        dif = (gi[b] - gs[b]).abs().max(dim=1).values
        bad = torch.nonzero(dif > 0).flatten().tolist()
        print('L%d B%d n%d elem %d: grouped i/s max %.3g, bad coords %d (first %s); single i/s %.3g; grouped_i vs single_i %.3g; grouped_s vs single_s %.3g'
              % (L, B, n, b, float(dif.max()), len(bad), bad[:8], float((g1 - g2).abs().max()), float((gi[b] - g1).abs().max()),
                 float((gs[b] - g2).abs().max())))
