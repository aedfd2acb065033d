"""Runs ONE training / inference path of the engine at its bench configuration, so a rocprofv3 kernel trace or PMC
pass over this process is attributable to that path (tools/profile_round.sh), and prints its HIP-event timing.

python tools/profile_paths.py <path> [--reps R]     (1 warm-up step + R timed steps; prints one JSON line)

Paths (BASELINE.json configs; F = 2 sum fan_in fan_out FLOP per coordinate):
  image_w2     5x256 d2 o1, 2^18 coords: forward_store + backward_stored (image_mse train kernels, W2 = 3F)
  sdf          5x256 d3 o1, 2^19 coords: forward_grad_store + seeded W3 from the kept forward (sdf kernels, 8F)
  video        5x512 d3 o3, 2^20 coords: forward_store + backward_stored (hidden 512 W2 = 3F)
  poisson      5x256 d2 o1, 512^2 grid: forward_laplace_store + laplace_backward_stored (W4s = 3 (1 + 2d) F = 15F)
  poisson_ref  5x256 d2 o1, 512^2 grid: the reference recipe's kernels in steady state: the shared Hessian node's
               forward (one 6-stream jet, kept, which also returns y and J: the module's jet forward from the third
               step on), ONE quadratic-form jet reverse (its backward); the same loss gradient as poisson (15F)
  w3_theta     5x256 d2 o1, 2^19 coords: W3 H v + theta-grads without a kept forward (6F)
  hypernet     32 x 4096 coords, 5x256 d2 o1 per-element weights: grouped stored forward + grouped reverse-only W2
               (the hypernetwork training kernels, W2 = 3F)
  hypernet_w3  the same batch: grouped W3 H v + theta-grads (second_order_batched, 6F); _loop = 32 single calls
  w1           5x256 d2 o1, 2^20 coords: the headline W1 launch (2F)
  w1x          the same on the split-bf16 kernel (w1x_kernel.hpp, precision mode bf16x6)
  w3_wide      5x512 d3 o1, 2^18 coords: W3 H v + theta-grads at hidden 512 (two-stream jet + wgrad, 6F)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PATHS = {  # name: (d, hidden, layers, o, n, work units of F)
    'image_w2': (2, 256, 3, 1, 1 << 18, 3),
    'image_w2x': (2, 256, 3, 1, 1 << 18, 3),  # the bf16x6 training leg: stored split-bf16 forward + reverse-only backward
    'sdf': (3, 256, 3, 1, 1 << 19, 8),
    'video': (3, 512, 3, 3, 1 << 20, 3),
    'poisson': (2, 256, 3, 1, 512 * 512, 15),
    'poisson_ref': (2, 256, 3, 1, 512 * 512, 15),
    'w3_theta': (2, 256, 3, 1, 1 << 19, 6),
    'hypernet': (2, 256, 3, 1, 32 * 4096, 3),
    'hypernet_np': (2, 256, 3, 1, 32 * 4096, 3),   # the same with SIREN_FLAG_NO_PERSIST (one workgroup per tile)
    'hypernet_w3': (2, 256, 3, 1, 32 * 4096, 6),   # grouped W3 H v + theta-grads over 32 per-element networks
    'hypernet_w3_loop': (2, 256, 3, 1, 32 * 4096, 6),  # the same as 32 single-network second_order calls
    'w1': (2, 256, 3, 1, 1 << 20, 2),
    'w1x': (2, 256, 3, 1, 1 << 20, 2),      # the split-bf16 W1 (precision mode bf16x6), same workload as w1
    'w0': (2, 256, 3, 1, 1 << 20, 1),       # the fp32 forward-only W0 (dense evaluation)
    'w0x': (2, 256, 3, 1, 1 << 20, 1),      # the split-bf16 forward-only W0
    'w3_wide': (3, 512, 3, 1, 1 << 18, 6),
    'video1024': (3, 1024, 3, 3, 1 << 18, 3),   # the layered path (train_video.py's width)
    'video1024_rc': (3, 1024, 3, 3, 1 << 18, 3),
    'fwd1024': (3, 1024, 3, 3, 1 << 18, 1),
}


def flop_per_coord(d, H, L, o):
    return 2 * (d * H + L * H * H + H * o)


def build_step(name, dev):
    from siren_amd.engine import SirenEngine
    from siren_amd.modules import FCBlock
    d, H, L, o, n, _ = PATHS[name]
    torch.manual_seed(0)
    net = FCBlock(d, o, L, H, outermost_linear=True, nonlinearity='sine')
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).to(dev)
    # SIREN_FLAGS (env): cfg.reserved flags for A/B runs (2 = SIREN_FLAG_NO_PERSIST)
    eng = SirenEngine(d, H, L, o, flags=2 if name == 'hypernet_np' else int(os.environ.get('SIREN_FLAGS', '0')))
    g = torch.Generator(device=dev).manual_seed(1)
    if name.startswith('hypernet_w3'):
        B = 32
        fb = flat[None].repeat(B, 1) + 1e-3 * torch.randn(B, flat.numel(), device=dev, generator=g)
        wsb = eng.pack_batched(fb, full=True)
        xb = torch.rand(B, n // B, d, device=dev, generator=g) * 2 - 1
        vb = torch.randn(B, n // B, d, device=dev, generator=g)
        if name == 'hypernet_w3':
            return lambda: eng.second_order_batched(wsb, xb, vb, want_theta=True)
        return lambda: [eng.second_order(wsb[b], xb[b], vb[b], want_theta=True) for b in range(B)]
    if name.startswith('hypernet'):
        B = 32
        fb = flat[None].repeat(B, 1) + 1e-3 * torch.randn(B, flat.numel(), device=dev, generator=g)
        wsb = eng.pack_batched(fb)
        xb = torch.rand(B, n // B, d, device=dev, generator=g) * 2 - 1
        gyb = torch.randn(B, n // B, o, device=dev, generator=g)
        def step():
            _, tws = eng.forward_store_batched(wsb, xb)
            eng.backward_stored_batched(wsb, xb, gyb, tws)
        return step
    ws = eng.pack(flat)
    if name.startswith('poisson'):
        from siren_amd import dataio
        x = dataio.get_mgrid(512).to(dev)
    else:
        x = torch.rand(n, d, device=dev, generator=g) * 2 - 1
    gy = torch.randn(n, o, device=dev, generator=g)
    if name == 'w1':
        return lambda: eng.forward_grad(ws, x)
    if name == 'w1x':
        wsx = eng.pack_split(flat)
        return lambda: eng.forward_grad_split(wsx, x)
    if name == 'w0':
        return lambda: eng.forward(ws, x)
    if name == 'w0x':
        wsx = eng.pack_split(flat)
        return lambda: eng.forward_split(wsx, x)
    if name == 'fwd1024':
        return lambda: eng.forward(ws, x)
    if name == 'video1024':  # the training split the module runs: stored forward, reverse-only backward
        def step():
            _, tws = eng.forward_store(ws, x)
            eng.backward_stored(ws, x, gy, tws)
        return step
    if name == 'video1024_rc':  # recompute backward (beyond SirenEngine.STORED_LAYERED_MAX_BYTES)
        def step():
            eng.forward(ws, x)
            eng.backward_params(ws, x, gy)
        return step
    if name == 'image_w2x':
        def step():
            wsx = eng.pack_split(flat)  # once per weight update, as SirenSplitFunction does
            _, tws = eng.forward_store_split(wsx, x)
            eng.backward_stored_split(wsx, x, gy, tws)
        return step
    if name in ('image_w2', 'video'):
        def step():
            _, tws = eng.forward_store(ws, x)
            eng.backward_stored(ws, x, gy, tws)
        return step
    if name == 'sdf':
        v = torch.randn(n, d, device=dev, generator=g)

        def step():
            _, _, kept = eng.forward_grad_store(ws, x)
            eng.second_order(ws, x, v, want_theta=True, gy=gy, kept=kept)
        return step
    if name in ('w3_theta', 'w3_wide'):
        v = torch.randn(n, d, device=dev, generator=g)
        return lambda: eng.second_order(ws, x, v, want_theta=True)
    gl = torch.randn(n, 1, device=dev, generator=g) / n
    if name == 'poisson':
        def step():
            _, tws = eng.forward_laplace_store(ws, x)
            eng.laplace_backward_stored(ws, x, gl, tws)
        return step
    if name == 'poisson_ref':
        es = []
        for i in range(d):
            e = torch.zeros(n, d, device=dev)
            e[:, i] = 1.
            es.append(e)

        G = torch.diag_embed(gl.expand(n, d))  # the summed cotangent of the shared Hessian node: glap * I

        def step():
            # the jet node's forward IS the shared Hessian node's sweep once the module has seen the recipe
            # (JetState.hessian): y, J, Hm and the kept jets in one launch (siren_hessian_ex)
            _, kept, _, _ = eng.hessian(ws, x, keep=True, want_yg=True)
            return eng.hessian_backward(ws, x, G, kept=kept)  # its ONE backward (third order): reverse-only jet
        return step
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('path', choices=sorted(PATHS))
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    dev = torch.device('cuda', 0)
    step = build_step(a.path, dev)
    step()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.reps):
        step()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    d, H, L, o, n, units = PATHS[a.path]
    flops = units * flop_per_coord(d, H, L, o) * n
    print(json.dumps({'path': a.path, 'n': n, 'steps_total': a.reps + 1, 'ms_per_step': round(ms, 4),
                      'flop_per_step': flops, 'tflops': round(flops / ms / 1e9, 2),
                      'frac_fp32_peak': round(flops / ms / 1e9 / 157.3, 4), 'mcoords_s': round(n / ms / 1e3, 3)}),
          flush=True)


if __name__ == '__main__':
    main()
