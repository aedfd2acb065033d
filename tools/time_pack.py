import sys, torch
sys.path.insert(0, '/root/repo')
from siren_amd.engine import SirenEngine
eng = SirenEngine(2, 256, 3, 1)
fb = torch.randn(32, eng.param_count, device='cuda') * 0.01
f1 = fb[0].contiguous()
for name, fn in (('pack_batched_32', lambda: eng.pack_batched(fb)), ('pack_1', lambda: eng.pack(f1))):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20): fn()
    b.record(); torch.cuda.synchronize()
    print(name, round(a.elapsed_time(b) / 20 * 1e3, 1), 'us')
