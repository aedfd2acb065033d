"""bench.py — the headline benchmark: Mcoords/s of the fused 5x256 SIREN forward + coordinate gradient (W1).

Workload (BASELINE.json configs[1]): SingleBVPNet defaults (d_in 2, hidden 256, 3 hidden layers, out 1, w0 30),
N = 2^20 uniform random 2-D coordinates per GPU per step (weak scaling), seed-0 reference-distributed weights.
One step = repack the weights (siren_pack) + ONE fused fwd+grad launch (siren_forward_grad: y and dPhi/dx)
over the GPU's whole batch, inputs resident in HBM. N GPUs: one process per GPU (torchrun), coordinates
sharded per rank with no collective on the data path (the W1 path has no exchange step); the timed region is
bracketed by barrier + synchronize and the max over ranks is used.

Also reported: roofline of the fused kernel (HIP events on the launch stream), the oracle's CPU restatement
timed on the host cores (cpu_baseline), a short W2 training-step rate, the PSNR of a 300-step image fit
against the reference's (tests/golden manifest), and per-config training / inference rates for the other
BASELINE configs (sdf = W3, 5x512 video = W2 at hidden 512, Poisson 512^2 = W4/W4s), all on the same JSON line.

Data-parallel training legs (every N, all ranks): BASELINE configs[2] (sdf, 5x256 d3, 2^19
coordinates per GPU resampled on the device every step, clip + Adam) and configs[3] (video, 5x512 d3 o3, 2^20
coordinates per GPU sampled from a 64x512x512 grid every step) with FusedAdam's ONE count-weighted all-reduce of
the flat gradient bucket over RCCL; the all-reduce is also timed alone.

python bench.py [--gpus N] [--steps K] [--warmup W] [--n COORDS] [--no-cpu] [--no-extra] [--no-dp]
With --gpus N > 1 outside torchrun, bench.py relaunches itself under torch.distributed.run (one process per GPU)
as a child process before touching the GPU.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 dense peak (measured 155)
HBM_PEAK_GBS = 8000.
H, LH, D_IN, D_OUT = 256, 3, 2, 1
F_PER_COORD = 2 * (D_IN * H + LH * H * H + H * D_OUT)   # 394,752 FLOP
W1_FLOP = 2 * F_PER_COORD                             # 789,504 FLOP / coord
REF_PSNR_DB = 39.13                                    # BASELINE.md §2 (reference, 300 steps, CPU)


def seed0_params(device):
    """Reference-distributed weights (modules.py:622-635 + nn.Linear bias init), generated on the host."""
    from siren_amd.modules import FCBlock
    torch.manual_seed(0)
    net = FCBlock(D_IN, D_OUT, LH, H, outermost_linear=True, nonlinearity='sine')
    return torch.cat([p.detach().reshape(-1) for p in net.parameters()]).to(device)


def _host_cpu():
    """CPU model name and physical core count of this host (/proc/cpuinfo), for the cpu_baseline record."""
    model, cores = None, set()
    try:
        phys = core = None
        for line in open('/proc/cpuinfo'):
            k, _, v = line.partition(':')
            k, v = k.strip(), v.strip()
            if k == 'model name' and model is None:
                model = v
            elif k == 'physical id':
                phys = v
            elif k == 'core id':
                core = v
            elif not k and phys is not None:
                cores.add((phys, core))
                phys = core = None
        if phys is not None:
            cores.add((phys, core))
    except OSError:
        pass
    return model, len(cores) or None


def _cpu_allotment():
    """CPUs this process may use: its affinity set, capped by the cgroup CPU quota (cpu.max) when one is set; the GPU
    box leases a share of a large host, and nproc / os.cpu_count() show the whole machine there."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota = None
    for path in ('/sys/fs/cgroup/cpu.max', '/sys/fs/cgroup/cpu/cpu.cfs_quota_us'):
        try:
            parts = open(path).read().split()
        except OSError:
            continue
        if path.endswith('cpu.max') and parts and parts[0] != 'max':
            quota = float(parts[0]) / float(parts[1])
        elif path.endswith('cfs_quota_us') and parts and int(parts[0]) > 0:
            period = float(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
            quota = float(parts[0]) / period
        break
    usable = affinity if quota is None else max(1, min(affinity, int(quota + 0.5)))
    return usable, affinity, quota


def cpu_baseline(sizes=(1 << 16, 1 << 18, 1 << 20), seconds=4.):
    """The oracle's torch restatement (reference op sequence + autograd gradient, i.e. the reference's CPU path) on
    the host cores at N = 2^16, 2^18, 2^20: at least one full pass and ~`seconds` of passes per
    size. value = the N = 2^20 rate (the headline workload's size)."""
    from oracle import siren_oracle as O
    threads_before = torch.get_num_threads()
    usable, affinity, quota = _cpu_allotment()
    torch.set_num_threads(usable)  # every CPU the lease gives this process (all host cores)
    torch.manual_seed(0)
    dims = [D_IN] + [H] * (LH + 1) + [D_OUT]
    params = []
    for i, (fi, fo) in enumerate(zip(dims[:-1], dims[1:])):
        bound = 1. / fi if i == 0 else np.sqrt(6. / fi) / 30.
        params += [((torch.rand(fo, fi) * 2 - 1) * bound), ((torch.rand(fo) * 2 - 1) / np.sqrt(fi))]
    rates, total = {}, 0.
    for n in sizes:
        x0 = torch.rand(1, n, D_IN) * 2 - 1
        done, t0 = 0, time.perf_counter()
        while True:
            x = x0.clone().requires_grad_(True)
            y = O.torch_forward(x, params)
            g = O.torch_gradient(y, x)
            _ = float(g.detach().sum())
            done += n
            el = time.perf_counter() - t0
            if el > seconds:
                break
        rates['n_2e%d' % (n.bit_length() - 1)] = round(done / el / 1e6, 4)
        total += el
    model, phys = _host_cpu()
    used = torch.get_num_threads()
    torch.set_num_threads(threads_before)
    return {'value': rates['n_2e%d' % (sizes[-1].bit_length() - 1)], 'unit': 'Mcoords/s',
            'cores': used, 'kind': 'port', 'rates_by_n': rates, 'cpu_model': model,
            'host_physical_cores': phys, 'lease_affinity_cpus': affinity,
            'lease_cgroup_cpu_quota': quota, 'all_lease_cpus_used': used == usable,
            'sample': 'N = %s coords, >= %.0f s each (%.1f s total): 5x256 d2 o1 fwd + autograd gradient, torch CPU '
                      'fp32 on %d threads = every CPU of the lease (affinity %d CPUs, cgroup quota %s)'
                      % ('/'.join('2^%d' % (n.bit_length() - 1) for n in sizes), seconds, total, used, affinity,
                         'none' if quota is None else '%.1f CPUs' % quota)}


def kernel_roofline(eng, ws, x, reps=10):
    """Average duration of the fused W1 launch from HIP events on the stream it is enqueued on."""
    st = torch.cuda.current_stream()
    y = torch.empty(x.shape[0], 1, device=x.device)
    gx = torch.empty_like(x)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st)
        eng.forward_grad(ws, x, out_y=y, out_gx=gx)
        b.record(st)
    torch.cuda.synchronize()
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    achieved = W1_FLOP * x.shape[0] / (ms * 1e-3) / 1e12
    return ms, achieved


PEAK_BF16_MFMA_TFLOPS = 2516.6     # MI355X dense bf16 MFMA peak (MI355X_MICROARCH.md; 16x the fp32 matrix rate)
# split-bf16 W1 (w1x_kernel.hpp): per coordinate, the 2 L hidden GEMMs (forward + reverse) run six bf16 products per
# fp32 K-step: 6 x 2 x (2 LH H^2) bf16 MFMA flops; the d_in / d_out layers are VALU
SPLIT_MFMA_FLOP = 6 * 2 * 2 * 3 * 256 * 256


def split_leg(eng, flat, x, steps, warmup):
    """The split-bf16 W1 (siren_pack_split + siren_forward_grad_split) on the headline workload: the same step (pack +
    one fused launch per step) timed the same way, its kernel duration from HIP events, its roofline against the
    dense bf16 MFMA peak, and its largest difference from the fp32 kernel on this batch. The headline value stays the
    fp32 kernel's (compute dtype >= the reference's fp32); this is the precision-mode alternative."""
    if not eng.split_supported:
        return None
    y = torch.empty(x.shape[0], 1, device=x.device)
    gx = torch.empty_like(x)

    def step():
        wsx = eng.pack_split(flat)
        eng.forward_grad_split(wsx, x, out_y=y, out_gx=gx)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    wsx = eng.pack_split(flat)
    st = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for a, b in ev:
        a.record(st)
        eng.forward_grad_split(wsx, x, out_y=y, out_gx=gx)
        b.record(st)
    torch.cuda.synchronize()
    kms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    ws = eng.pack(flat)
    y32, g32 = eng.forward_grad(ws, x)
    achieved_bf16 = SPLIT_MFMA_FLOP * x.shape[0] / (kms * 1e-3) / 1e12
    # the forward-only W0 on the same image (dense evaluation), beside the fp32 W0 kernel
    yf = torch.empty(x.shape[0], 1, device=x.device)
    fwd = {}
    for name, fn in (('fp32', lambda: eng.forward(ws, x, out=yf)), ('split', lambda: eng.forward_split(wsx, x, out=yf))):
        fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            a.record(st)
            fn()
            b.record(st)
        torch.cuda.synchronize()
        fwd[name] = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    return {'value': round(x.shape[0] * steps / el / 1e6, 3), 'unit': 'Mcoords/s',
            'ms_per_step': round(el / steps * 1e3, 4), 'kernel_ms': round(kms, 4),
            'dtype': 'bf16x6 (fp32 operands split exactly into bf16 hi/mid/lo, 6 products per K-step, fp32 accumulate)',
            'fp32_equiv_tflops': round(W1_FLOP * x.shape[0] / (kms * 1e-3) / 1e12, 2),
            'roofline': {'bound': 'mfma', 'achieved': round(achieved_bf16, 2), 'peak': PEAK_BF16_MFMA_TFLOPS,
                         'unit': 'TFLOP/s', 'frac': round(achieved_bf16 / PEAK_BF16_MFMA_TFLOPS, 4),
                         'flop_per_coord': SPLIT_MFMA_FLOP},
            'forward_w0': {'split_mcoords_s': round(x.shape[0] / fwd['split'] / 1e3, 2),
                           'fp32_mcoords_s': round(x.shape[0] / fwd['fp32'] / 1e3, 2),
                           'split_kernel_ms': round(fwd['split'], 4), 'fp32_kernel_ms': round(fwd['fp32'], 4),
                           'bf16_frac': round(SPLIT_MFMA_FLOP / 2 * x.shape[0] / (fwd['split'] * 1e-3) / 1e12
                                              / PEAK_BF16_MFMA_TFLOPS, 4)},
            'max_abs_dy_vs_fp32_kernel': float((y - y32).abs().max()),
            'max_abs_dgrad_vs_fp32_kernel': float((gx - g32).abs().max()),
            'parity': 'tests/test_gpu_split.py: G1/G2 reference goldens vs fp64 within the fp32 kernel\'s error'}


# the bf16x6 W2 unit per coordinate on the bf16 pipe (stored split): forward (LH H^2), reverse (LH H^2) and the hidden
# wgrad (LH H^2), six products each
SPLIT_TRAIN_MFMA_FLOP = 6 * 2 * 3 * 3 * 256 * 256


def split_train_leg(device, fp32_rate, n=1 << 18):
    """image_mse training with precision='bf16x6' (the drop-in module, Adam included) at the image_w2 size, beside the
    fp32 step's rate, with the split kernels' durations from a trace-free HIP-event timing of one backward."""
    from siren_amd.engine import SirenEngine
    rate = train_step_rate(device, n=n, precision='bf16x6')
    eng = SirenEngine(2, 256, 3, 1, 30., 30., True)
    torch.manual_seed(0)
    from siren_amd.modules import FCBlock
    net = FCBlock(2, 1, 3, 256, outermost_linear=True, nonlinearity='sine')
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).to(device)
    x = torch.rand(n, 2, device=device) * 2 - 1
    gy = torch.randn(n, 1, device=device) / n
    st = torch.cuda.current_stream()
    wsx = eng.pack_split(flat)
    times = {}
    _, tws = eng.forward_store_split(wsx, x)
    for name, fn in (('forward_split', lambda: eng.forward_store_split(wsx, x)),
                     ('backward_split', lambda: eng.backward_stored_split(wsx, x, gy, tws))):
        fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            a.record(st)
            fn()
            b.record(st)
        torch.cuda.synchronize()
        times[name] = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    unit_ms = times['forward_split'] + times['backward_split']
    achieved = SPLIT_TRAIN_MFMA_FLOP * n / (unit_ms * 1e-3) / 1e12
    return {'value': round(rate, 3), 'unit': 'Mcoords/s', 'fp32_value': fp32_rate,
            'speedup_vs_fp32': round(rate / fp32_rate, 3) if fp32_rate else None,
            'forward_ms': round(times['forward_split'], 4), 'backward_ms': round(times['backward_split'], 4),
            'roofline': {'bound': 'mfma', 'achieved': round(achieved, 2), 'peak': PEAK_BF16_MFMA_TFLOPS,
                         'unit': 'TFLOP/s', 'frac': round(achieved / PEAK_BF16_MFMA_TFLOPS, 4),
                         'flop_per_coord': SPLIT_TRAIN_MFMA_FLOP,
                         'note': 'forward + backward launches (split forward with stores, split reverse, bf16x6 wgrad, edge, reduce)'},
            'parity': 'tests/test_gpu_split.py: G1 image_mse theta-grads vs fp64 within the fp32 pipeline\'s error'}


HEADLINE_KERNEL = 'w1_kernel<3,640>'   # MODE_W1 | MODE_O1S | MODE_D(2), as tools/pmc_summary.py shortens it
PMC_FILE = os.path.join(ROOT, 'profiles', 'pmc_headline.json')


def pmc_traffic(n):
    """HBM bytes per launch of the headline kernel from the committed rocprofv3 PMC summary
    (profiles/pmc_headline.json: tools/gpu_round.sh's FETCH_SIZE / WRITE_SIZE passes through tools/pmc_summary.py),
    if it holds this kernel at this N AND was collected on a library built from the sources of this tree (its
    `source_hash` stamp equals __graft_entry__._source_hash()); else None — a profile of an older kernel is never
    reported as this one's traffic. Returns (bytes or None, provenance note)."""
    try:
        rec = json.load(open(PMC_FILE))
    except Exception:
        return None, 'no profiles/pmc_headline.json'
    import __graft_entry__
    if rec.get('source_hash') != __graft_entry__._source_hash():
        return None, 'profiles/pmc_headline.json was collected on another build (source_hash %s)' % (
            str(rec.get('source_hash'))[:12])
    k = rec.get('kernels', {}).get(HEADLINE_KERNEL)
    if k and rec.get('n') == n and 'hbm_bytes_per_launch' in k:
        return round(k['hbm_bytes_per_launch']), 'profiles/pmc_headline.json (source_hash %s, FETCH_SIZE x2 + ' \
            'WRITE_SIZE per MI355X_MICROARCH.md)' % rec['source_hash'][:12]
    return None, 'profiles/pmc_headline.json lacks %s at n=%d' % (HEADLINE_KERNEL, n)


def train_step_rate(device, n=1 << 18, steps=10, warmup=3, precision='fp32'):
    """W2: image_mse training steps (fused forward, fused backward + MFMA wgrad, Adam) in Mcoords/s. precision
    'bf16x6': the split-bf16 leg (split W0 forward, siren_backward_split: split-bf16 recompute + reverse, bf16x6 wgrad)."""
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(0)
    model = SingleBVPNet(verbose=False, jet=False, precision=precision).to(device)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    x = torch.rand(1, n, 2, device=device) * 2 - 1
    gt = torch.sin(5 * x[..., :1])
    def step():
        out = model({'coords': x})
        loss = ((out['model_out'] - gt) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
    for _ in range(warmup):  # Adam state, allocator pools
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return n * steps / (time.perf_counter() - t0) / 1e6


def reference_laplace(y, x):
    """diff_operators.laplace as the reference writes it (diff_operators.py:27-43), restated: gradient with
    create_graph, then divergence = one create_graph autograd.grad per input dimension."""
    grad = torch.autograd.grad(y, [x], grad_outputs=torch.ones_like(y), create_graph=True)[0]
    div = 0.
    for i in range(grad.shape[-1]):
        div += torch.autograd.grad(grad[..., i], x, torch.ones_like(grad[..., i]), create_graph=True)[0][..., i:i + 1]
    return div


def config_rates(device, steps=10, warmup=3):
    """Secondary per-config rates (BASELINE.json configs[2..4]), one GPU, drop-in API end to end (model ->
    loss_functions -> backward -> Adam), inputs resident on the device. Mcoords/s per GPU."""
    from siren_amd.modules import SingleBVPNet
    from siren_amd import loss_functions as LF
    from siren_amd import dataio
    from siren_amd.engine import SirenEngine
    res = {}

    def rate(model, x, loss_fn, n):
        opt = torch.optim.Adam(model.parameters(), lr=1e-4)

        def step():
            out = model({'coords': x})
            total = sum(v.mean() for v in loss_fn(out).values())
            opt.zero_grad()
            total.backward()
            opt.step()
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        return round(n * steps / (time.perf_counter() - t0) / 1e6, 3)

    # configs[2]: sdf (W3 training: on/off-surface sphere batch), 5x256 d3, 2^19 coords per GPU
    torch.manual_seed(0)
    m = SingleBVPNet(in_features=3, verbose=False).to(device)
    inp, gt_sdf = dataio.sphere_sdf_batch(1 << 18, device=device)  # 2^18 on + 2^18 off surface = 2^19
    n = inp['coords'].shape[1]
    res['sdf_5x256_d3_train_mcoords_s'] = rate(m, inp['coords'], lambda o: LF.sdf(o, gt_sdf), n)
    # configs[2] as the reference's loop runs it (train_sdf.py: PointCloud resampled every step, clip_grad):
    # device sampler (siren_sample_sdf) + fused clip + Adam (siren_adam_step) inside the timed step
    from siren_amd.optim import FusedAdam
    g = torch.Generator().manual_seed(0)
    d = torch.randn(1 << 20, 3, generator=g, dtype=torch.float64)
    d = d / d.norm(dim=-1, keepdim=True)
    pcd = dataio.PointCloud(points=torch.cat([d * 0.5, d], 1).numpy(), on_surface_points=1 << 18, device=device)
    torch.manual_seed(0)
    m = SingleBVPNet(in_features=3, verbose=False).to(device)
    fopt = FusedAdam(m.parameters(), lr=1e-4, max_norm=1.)

    def sdf_step(i):
        inp_i, gt_i = pcd.sample(i)
        out = m({'coords': inp_i['coords'][None]})
        total = sum(v.mean() for v in LF.sdf(out, {k: v[None] for k, v in gt_i.items()}).values())
        fopt.zero_grad()
        total.backward()
        fopt.step()
    for i in range(warmup):
        sdf_step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        sdf_step(warmup + i)
    torch.cuda.synchronize()
    res['sdf_5x256_d3_train_device_sampling_fused_adam_mcoords_s'] = round(
        (1 << 19) * steps / (time.perf_counter() - t0) / 1e6, 3)
    # the per-step kernels alone (HBM-bound): sampler algorithmic bytes = k (index gather: 24 B read) + 2k rows
    # written (coords 12 + normals 12 + sdf 4 B); Adam = 28 B / parameter (g, m, v, p read; m, v, p written)
    st = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record(st)
    for i in range(20):
        pcd.sample(100 + i)
    ev[1].record(st)
    ev[2].record(st)
    for _ in range(20):
        fopt.step()
    ev[3].record(st)
    torch.cuda.synchronize()
    k = 1 << 18
    ms_s, ms_a = ev[0].elapsed_time(ev[1]) / 20, ev[2].elapsed_time(ev[3]) / 20
    P = sum(p.numel() for p in m.parameters())
    # (event spans over 20 back-to-back calls: host-launch-inclusive; the kernel-only durations are in the
    # rocprofv3 summary, profiles/r01_step_kernels_stats.csv)
    res['step_kernels'] = {'sample_sdf_us_per_call': round(ms_s * 1e3, 2),
                           'sample_sdf_bytes': 24 * k + 2 * k * 28,
                           'clip_adam_us_per_call': round(ms_a * 1e3, 2),
                           'clip_adam_bytes': 28 * P, 'params': P}
    # §8f row 2: batched hypernetwork weights, a meta-batch of 32 64x64 images (grouped W1 launch over the batch)
    eng_b = SirenEngine(2, 256, 3, 1)
    flat_b = torch.randn(32, eng_b.param_count, device=device) * 0.01
    xb = torch.rand(32, 4096, 2, device=device) * 2 - 1
    wsb = eng_b.pack_batched(flat_b)
    for _ in range(warmup):
        eng_b.forward_grad_batched(wsb, xb)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng_b.forward_grad_batched(wsb, xb)
    torch.cuda.synchronize()
    res['hypernet_b32x4096_grouped_w1_mcoords_s'] = round(32 * 4096 * steps / (time.perf_counter() - t0) / 1e6, 3)
    # the hypernetwork training kernels: the per-step batched pack (the hypernetwork predicts new weights every step),
    # grouped stored forward + grouped reverse-only W2 (3F per coordinate)
    gyb = torch.randn(32, 4096, 1, device=device)

    def hyper_w2():
        ws_step = eng_b.pack_batched(flat_b)
        _, tws = eng_b.forward_store_batched(ws_step, xb)
        eng_b.backward_stored_batched(ws_step, xb, gyb, tws)
    for _ in range(warmup):
        hyper_w2()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        hyper_w2()
    torch.cuda.synchronize()
    res['hypernet_b32x4096_grouped_w2_train_mcoords_s'] = round(32 * 4096 * steps / (time.perf_counter() - t0) / 1e6, 3)
    # configs[3] (video, 5x512 d3 o3, 2^20 coordinates per GPU sampled from a 64x512x512 volume): dp_train
    # configs[4]: Poisson on a 512^2 grid: laplace_mse training (W4 + W4s) and W4 inference (y, grad, Laplacian)
    torch.manual_seed(0)
    m = SingleBVPNet(verbose=False).to(device)
    grid = dataio.get_mgrid(512)[None].to(device)
    n = grid.shape[1]
    lap_gt = torch.sin(4 * grid[..., :1])
    res['poisson_512sq_laplace_mse_train_mcoords_s'] = rate(m, grid, lambda o: LF.laplace_mse(o, {'laplace': lap_gt}), n)
    # the same loss through the reference's own op sequence (diff_operators.py:27-43: gradient, then one create_graph
    # autograd.grad per input dimension) instead of siren_amd's fused laplace(): d Hessian-vector-product nodes
    # whose backward is the third-order mixed-jet kernel (siren_hvp_backward)
    torch.manual_seed(0)
    m = SingleBVPNet(verbose=False).to(device)
    res['poisson_512sq_reference_recipe_laplace_mse_train_mcoords_s'] = rate(
        m, grid, lambda o: {'laplace_loss': ((reference_laplace(o['model_out'], o['model_in']) - lap_gt) ** 2).mean()},
        n)
    eng = SirenEngine(2, 256, 3, 1)
    ws = eng.pack(seed0_params(device))
    x2 = grid[0].contiguous()
    for _ in range(warmup):
        eng.forward_laplace(ws, x2, True, True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.forward_laplace(ws, x2, True, True)
    torch.cuda.synchronize()
    res['poisson_512sq_w4_y_grad_laplacian_mcoords_s'] = round(n * steps / (time.perf_counter() - t0) / 1e6, 3)
    return res


def dp_train_rates(device, world, rank, steps=5, warmup=2):
    """Data-parallel training steps at every N (weak scaling: a fixed per-GPU batch), the reference's loop semantics
    (training.py:72-104: forward, loss means, backward, all-reduce, clip, Adam) with FusedAdam's single count-
    weighted all-reduce of the flat gradient bucket. Returns {config: {...}}; rates are whole-job Mcoords/s from the
    max over ranks of the timed region."""
    import torch.distributed as dist
    from siren_amd.modules import SingleBVPNet
    from siren_amd import loss_functions as LF
    from siren_amd import dataio
    from siren_amd.optim import FusedAdam
    from siren_amd import distributed as sd
    res = {}

    def timed(step_fn, n_local, opt):
        for i in range(warmup):
            step_fn(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            step_fn(warmup + i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        ar_us = None
        if world > 1:
            t = torch.tensor([el], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
            # the bucket all-reduce alone (same size and backend), HIP events on the current stream
            st = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                dist.all_reduce(opt.bucket)
            torch.cuda.synchronize()
            e0.record(st)
            for _ in range(20):
                dist.all_reduce(opt.bucket)
            e1.record(st)
            torch.cuda.synchronize()
            ar_us = round(e0.elapsed_time(e1) / 20 * 1e3, 2)
        return {'mcoords_s': round(world * n_local * steps / el / 1e6, 3), 'ms_per_step': round(el / steps * 1e3, 3),
                'coords_per_gpu': n_local, 'allreduce_us': ar_us, 'bucket_bytes': int(opt.bucket.numel() * 4),
                'steps': steps}

    # configs[2]: sdf, 5x256 d3, 2^18 on + 2^18 off surface per GPU, device PointCloud resampled every step,
    # clip_grad=True (train_sdf.py:57-60)
    g = torch.Generator().manual_seed(0)
    d = torch.randn(1 << 20, 3, generator=g, dtype=torch.float64)
    d = d / d.norm(dim=-1, keepdim=True)
    pcd = dataio.PointCloud(points=torch.cat([d * 0.5, d], 1).numpy(), on_surface_points=1 << 18, device=device)
    torch.manual_seed(0)
    m = SingleBVPNet(in_features=3, verbose=False).to(device)
    sd.broadcast_parameters(m)
    opt = FusedAdam(m.parameters(), lr=1e-4, max_norm=1.)

    def sdf_step(i):
        inp, gt = pcd.sample(i * world + rank)  # each rank its own draw
        out = m({'coords': inp['coords'][None]})
        total = sum(v.mean() for v in LF.sdf(out, {k: v[None] for k, v in gt.items()}).values())
        opt.zero_grad()
        total.backward()
        if world > 1:
            opt.allreduce_grad(world, inp['coords'].shape[0])
        opt.step()
    res['sdf_5x256_d3'] = timed(sdf_step, 1 << 19, opt)
    del m, opt, pcd
    # configs[3]: video, 5x512 d3 o3 (image_mse), 2^20 coordinates per GPU sampled every step from the 64x512x512
    # grid of a synthetic video (dataio.py:655-673 Implicit3DWrapper, sample_fraction < 1: randint rows)
    mgrid = dataio.get_mgrid((64, 512, 512), dim=3).to(device)
    vid = dataio.synthetic_video(mgrid)
    torch.manual_seed(0)
    m = SingleBVPNet(in_features=3, out_features=3, hidden_features=512, verbose=False).to(device)
    sd.broadcast_parameters(m)
    opt = FusedAdam(m.parameters(), lr=1e-4)
    gen = torch.Generator(device=device).manual_seed(100 + rank)
    nv = 1 << 20

    def video_step(i):
        idx = torch.randint(0, mgrid.shape[0], (nv,), device=device, generator=gen)
        out = m({'coords': mgrid[idx][None]})
        total = LF.image_mse(None, out, {'img': vid[idx][None]})['img_loss'].mean()
        opt.zero_grad()
        total.backward()
        if world > 1:
            opt.allreduce_grad(world, nv)
        opt.step()
    res['video_5x512_d3o3'] = timed(video_step, nv, opt)
    # the same loop at train_video.py's own width (hidden_features=1024, experiment_scripts/train_video.py): the
    # layered path (layered.hip: rocBLAS layer GEMMs + fused epilogues, stored-forward split)
    torch.manual_seed(0)
    m = SingleBVPNet(in_features=3, out_features=3, hidden_features=1024, verbose=False).to(device)
    sd.broadcast_parameters(m)
    opt = FusedAdam(m.parameters(), lr=1e-4)
    res['video_5x1024_d3o3'] = timed(video_step, nv, opt)
    del m, opt, mgrid, vid
    torch.cuda.empty_cache()
    return res


PATH_UNITS = {'w1': 2, 'image_w2': 3, 'sdf': 8, 'video': 3, 'video1024': 3, 'poisson': 15, 'poisson_ref': 15,
              'hypernet': 3}


def path_rooflines(rates):
    """Per-config roofline for the training paths: the MFMA fraction of the path's algorithmic flops (SURVEY.md §8a
    work units) at the rate measured live in this run (whole step: kernels + loss / optimizer / sampling ops), and
    from the committed per-path profile (profiles/pmc_<path>.json, tools/profile_round.sh: rocprofv3 kernel time,
    FETCH_SIZE / WRITE_SIZE HBM bytes per step and the kernels' I/O-contract bytes)."""
    out = {}
    for key, mc in rates.items():
        if mc is None:
            continue
        path = key.split('@')[0]  # 'image_w2@n2p20': the same path at another N (same kernels, same profile)
        try:
            rec = json.load(open(os.path.join(ROOT, 'profiles', 'pmc_%s.json' % path)))
        except (OSError, ValueError):
            rec = None
        if rec is None:
            continue
        c = rec['config']
        F = 2 * (c['d_in'] * c['hidden'] + c['hidden_layers'] * c['hidden'] ** 2 + c['hidden'] * c['d_out'])
        ach = PATH_UNITS[path] * F * mc * 1e6 / 1e12
        out[key] = {'bound': 'mfma', 'unit': 'TFLOP/s', 'peak': PEAK_FP32_MFMA_TFLOPS,
                     'flop_per_coord': PATH_UNITS[path] * F, 'achieved_step': round(ach, 2),
                     'frac_step': round(ach / PEAK_FP32_MFMA_TFLOPS, 4),
                     'frac_kernels_rocprof': rec.get('mfma_frac_of_kernel_time'),
                     'traffic_bytes_per_step': rec.get('hbm_bytes_per_step'),
                     'io_bytes_per_step': rec.get('io_bytes_per_step'), 'profiled_n': rec.get('n'),
                     'profile': 'profiles/pmc_%s.json' % path}
    return out


def psnr_fit(device, steps=300):
    """Config-1 fit (256^2 synthetic image, full batch, Adam lr 1e-4, image_mse) on the fused engine."""
    from siren_amd.modules import SingleBVPNet
    from siren_amd import dataio
    torch.manual_seed(0)
    model = SingleBVPNet(verbose=False, jet=False).to(device)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    grid = dataio.get_mgrid(256)[None].to(device)
    img = dataio.synthetic_image(grid)
    t0 = time.perf_counter()
    for _ in range(steps):
        out = model({'coords': grid})
        loss = ((out['model_out'] - img) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
    with torch.no_grad():
        pred = model({'coords': grid})['model_out']
    torch.cuda.synchronize()
    return dataio.psnr(pred, img), time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--n', type=int, default=1 << 20, help='coordinates per GPU per step')
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--no-extra', action='store_true')
    ap.add_argument('--no-dp', action='store_true', help='skip the data-parallel training legs')
    args = ap.parse_args()

    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        # one process per GPU: relaunch under torchrun as a CHILD process, before anything touches the GPU
        s = socket.socket()
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(args.gpus),
               '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # one GPU per rank over RCCL ("nccl"); SIREN_DIST_BACKEND=gloo with more ranks than GPUs is a rehearsal mode
    # (ranks share devices round-robin) for checking the multi-rank code path on a 1-GPU box
    ndev = max(1, torch.cuda.device_count())
    dev_idx = local if local < ndev else local % ndev
    if world > 1:
        torch.cuda.set_device(dev_idx)
        dist.init_process_group(os.environ.get('SIREN_DIST_BACKEND', 'nccl'))
    device = torch.device('cuda', dev_idx)

    import __graft_entry__
    __graft_entry__.build()
    from siren_amd.engine import SirenEngine
    eng = SirenEngine(D_IN, H, LH, D_OUT)
    flat = seed0_params(device)
    g = torch.Generator(device='cpu').manual_seed(1000 + rank)
    x = (torch.rand(args.n, D_IN, generator=g) * 2 - 1).to(device)
    y = torch.empty(args.n, D_OUT, device=device)
    gx = torch.empty_like(x)

    def step():
        ws = eng.pack(flat)
        eng.forward_grad(ws, x, out_y=y, out_gx=gx)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    value = world * args.n * args.steps / el / 1e6

    ws = eng.pack(flat)
    kms, achieved = kernel_roofline(eng, ws, x)
    n_ranks = dist.get_world_size() if world > 1 else 1  # ranks the process group (RCCL) initialised
    del y, gx, ws
    split = split_leg(eng, flat, x, args.steps, args.warmup) if rank == 0 else None
    dp = None if args.no_dp else dp_train_rates(device, n_ranks, rank)
    extra = {}
    if rank == 0 and not args.no_extra:
        extra['w2_image_mse_train_mcoords_s'] = round(train_step_rate(device), 3)
        if split is not None:  # the opt-in bf16x6 training leg beside the fp32 one
            split['train_w2_image_mse'] = split_train_leg(device, extra['w2_image_mse_train_mcoords_s'])
        # config 2's own N (2^20 coordinates per step) beside the 2^18 leg the per-path profile is taken at
        extra['w2_image_mse_train_n2p20_mcoords_s'] = round(train_step_rate(device, n=1 << 20), 3)
        extra['configs'] = config_rates(device)
        cr, dpr = extra['configs'], dp or {}
        extra['roofline_by_path'] = path_rooflines({
            'image_w2': extra['w2_image_mse_train_mcoords_s'],
            'image_w2@n2p20': extra['w2_image_mse_train_n2p20_mcoords_s'],  # config 2's own N
            'sdf': dpr.get('sdf_5x256_d3', {}).get('mcoords_s') if n_ranks == 1 else None,
            'video': dpr.get('video_5x512_d3o3', {}).get('mcoords_s') if n_ranks == 1 else None,
            'video1024': dpr.get('video_5x1024_d3o3', {}).get('mcoords_s') if n_ranks == 1 else None,
            'poisson': cr['poisson_512sq_laplace_mse_train_mcoords_s'],
            'poisson_ref': cr['poisson_512sq_reference_recipe_laplace_mse_train_mcoords_s'],
            'hypernet': cr['hypernet_b32x4096_grouped_w2_train_mcoords_s']})
        p, secs = psnr_fit(device)
        extra['psnr_db'] = {'value': round(p, 3), 'reference_cpu': REF_PSNR_DB, 'steps': 300,
                            'fit_seconds': round(secs, 2)}
    cpu = None
    if rank == 0 and n_ranks == 1 and not args.no_cpu:
        cpu = cpu_baseline()

    if rank == 0:
        traffic, traffic_src = pmc_traffic(args.n)
        line = {
            'metric': 'Mcoords/sec fwd+∇ (5×256 SIREN) at 1/2/4/8 MI355X; PSNR vs ref',
            'value': round(value, 3), 'unit': 'Mcoords/s', 'n_gpus': n_ranks, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(el / args.steps * 1e3, 4), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic',
            'config': {'workload': 'W1 fused fwd+grad, SingleBVPNet 5x256 (d_in 2, 3 hidden, out 1, w0 30), '
                                   'N=%d random coords per GPU per step' % args.n,
                       'coords_per_gpu': args.n, 'parallelism': 'dp%d' % n_ranks},
            'roofline': {'bound': 'mfma', 'achieved': round(achieved, 3), 'peak': PEAK_FP32_MFMA_TFLOPS,
                         'unit': 'TFLOP/s', 'frac': round(achieved / PEAK_FP32_MFMA_TFLOPS, 4),
                         'traffic': traffic, 'traffic_source': traffic_src, 'kernel_ms': round(kms, 4),
                         'flop_per_coord': W1_FLOP},
            'cpu_baseline': cpu,
            'split_bf16x6': split,
            'dp_train': dp,
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
