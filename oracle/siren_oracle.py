"""CPU restatement of the reference's SIREN hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only as the
checker / the timed CPU baseline. The product path (siren_amd) never imports it and has no CPU fallback.

Two restatements of xvdp/siren (/root/reference, read as text only):

* numpy fp64, analytic (the oracle proper):
    forward            modules.py:16-25 (BatchLinear: x W^T, += b), modules.py:32-34 (Sine: sin(30 z)),
                       modules.py:89-94 / 143-160 (FCBlock / SingleBVPNet: outermost layer linear),
                       ipynb SineLayer/Siren (first_omega_0 / hidden_omega_0, optional final sine)
    forward_grad       diff_operators.py:39-43 gradient = autograd.grad(y, x, grad_outputs=gy) -> reverse sweep
    forward_laplace    diff_operators.py:27-36 laplace = divergence(gradient) -> second-order forward Taylor
* torch (CPU), the reference's op sequence with autograd (torch_forward): used for the loss theta-gradients
  (loss_functions.py:8-12 image_mse, :84-89 gradients_mse, :104-109 laplace_mse, :214-238 sdf) and as the
  "reference CPU path" that bench.py times on the GPU box's host cores (cpu_baseline, kind "port").

* per-step work: sample_sdf restates the device PointCloud sampler (dataio.py:420-442)
  with the engine's counter RNG — bit-exact, but "parity unpinned" against the reference, whose np.random draws
  have no golden; adam_steps restates torch.optim.Adam + clip_grad_norm_ (training.py:17, 98-104), pinned on the
  GPU box against torch's own implementation (tests/test_gpu_step.py).

Parity is pinned: tests/test_oracle.py checks both restatements against the golden vectors that
tests/golden/make_golden.py produced by running the reference itself.
"""
import numpy as np

# ----------------------------------------------------------------------------------------------------------
# parameter plumbing (flat buffer in nn.Linear / state_dict order, include/siren_amd.h)
# ----------------------------------------------------------------------------------------------------------


def layers_from_state(sd, prefix='w_'):
    """[(W, b), ...] from a state dict (or fixture dict with key prefix) keyed net.net.{i}.0.{weight,bias}."""
    out, i = [], 0
    while True:
        kw = '%snet.net.%d.0.weight' % (prefix, i)
        if kw not in sd:
            break
        out.append((np.asarray(sd[kw]), np.asarray(sd['%snet.net.%d.0.bias' % (prefix, i)])))
        i += 1
    return out


def flatten(layers):
    return np.concatenate([np.concatenate([W.reshape(-1), b.reshape(-1)]) for W, b in layers])


def unflatten(flat, d_in, hidden, n_hidden, d_out):
    dims = [d_in] + [hidden] * (n_hidden + 1) + [d_out]
    layers, off = [], 0
    for fi, fo in zip(dims[:-1], dims[1:]):
        W = flat[off:off + fo * fi].reshape(fo, fi)
        off += fo * fi
        b = flat[off:off + fo]
        off += fo
        layers.append((W, b))
    assert off == flat.size
    return layers


# ----------------------------------------------------------------------------------------------------------
# numpy fp64 analytic restatement
# ----------------------------------------------------------------------------------------------------------


def _omegas(n_layers, omega_first, omega_hidden):
    return [omega_first] + [omega_hidden] * (n_layers - 1)


def forward(x, layers, omega_first=30., omega_hidden=30., outermost_linear=True):
    """Phi(x) in fp64 (modules.py:16-34, 89-94)."""
    a = np.asarray(x, np.float64)
    om = _omegas(len(layers), omega_first, omega_hidden)
    for li, (W, b) in enumerate(layers):
        z = a @ np.asarray(W, np.float64).T + np.asarray(b, np.float64)
        last = li == len(layers) - 1
        a = z if (last and outermost_linear) else np.sin(om[li] * z)
    return a


def forward_grad(x, layers, gy=None, omega_first=30., omega_hidden=30., outermost_linear=True):
    """(y, gx) with gx = sum_j gy_j dy_j/dx (gy=None: ones) — what autograd.grad(y, x, gy) returns
    (diff_operators.py:39-43), by an explicit reverse sweep in fp64."""
    a = np.asarray(x, np.float64)
    om = _omegas(len(layers), omega_first, omega_hidden)
    cos_stack = []
    for li, (W, b) in enumerate(layers):
        z = a @ np.asarray(W, np.float64).T + np.asarray(b, np.float64)
        last = li == len(layers) - 1
        if last and outermost_linear:
            a = z
            cos_stack.append(None)
        else:
            a = np.sin(om[li] * z)
            cos_stack.append(om[li] * np.cos(om[li] * z))
    y = a
    g = np.ones_like(y) if gy is None else np.asarray(gy, np.float64)
    for li in range(len(layers) - 1, -1, -1):
        if cos_stack[li] is not None:
            g = g * cos_stack[li]
        g = g @ np.asarray(layers[li][0], np.float64)
    return y, g


def forward_laplace(x, layers, omega_first=30., omega_hidden=30., outermost_linear=True):
    """(y, grad, lap) for d_out == 1: value, gradient and Laplacian sum_i d2y/dx_i^2 (diff_operators.py:27-36)
    by forward-mode Taylor propagation of (value, d tangents, Laplacian) in fp64."""
    x = np.asarray(x, np.float64)
    n, d = x.shape
    om = _omegas(len(layers), omega_first, omega_hidden)
    v = x
    t = np.broadcast_to(np.eye(d)[None], (n, d, d)).copy()  # t[c, i, k] = d v_k / d x_i
    s = np.zeros_like(x)                                     # s[c, k]   = sum_i d2 v_k / d x_i^2
    for li, (W, b) in enumerate(layers):
        W = np.asarray(W, np.float64)
        z = v @ W.T + np.asarray(b, np.float64)
        tz = t @ W.T
        sz = s @ W.T
        last = li == len(layers) - 1
        if last and outermost_linear:
            v, t, s = z, tz, sz
        else:
            w = om[li]
            sn, cs = np.sin(w * z), np.cos(w * z)
            v = sn
            t = (w * cs)[:, None, :] * tz
            s = w * cs * sz - w * w * sn * np.sum(tz * tz, axis=1)
    assert v.shape[1] == 1, 'forward_laplace restates the o == 1 case'
    return v, t[:, :, 0], s


# ----------------------------------------------------------------------------------------------------------
# torch restatement (reference op sequence + autograd), CPU
# ----------------------------------------------------------------------------------------------------------


def torch_forward(x, params, omega_first=30., omega_hidden=30., outermost_linear=True):
    """The reference's op sequence on torch tensors: x.matmul(W^T), += b (modules.py:23-24), sin(w*z)
    (modules.py:34). `params` is the list [W0, b0, W1, b1, ...]."""
    a = x
    nl = len(params) // 2
    for li in range(nl):
        W, b = params[2 * li], params[2 * li + 1]
        z = a.matmul(W.permute(1, 0))
        z = z + b.unsqueeze(-2)
        last = li == nl - 1
        if not (last and outermost_linear):
            z = (omega_first if li == 0 else omega_hidden) * z
            z = z.sin()
        a = z
    return a


def torch_gradient(y, x):
    import torch
    return torch.autograd.grad(y, [x], grad_outputs=torch.ones_like(y), create_graph=True)[0]


def torch_laplace(y, x):
    import torch
    g = torch_gradient(y, x)
    div = 0.
    for i in range(g.shape[-1]):
        div = div + torch.autograd.grad(g[..., i], x, torch.ones_like(g[..., i]), create_graph=True)[0][..., i:i + 1]
    return div


def torch_loss_terms(name, y, x, gt):
    """Loss terms as in loss_functions.py (image_mse 8-12, gradients_mse 84-89, laplace_mse 104-109, sdf 214-238)."""
    import torch
    import torch.nn.functional as F
    if name == 'image_mse':
        return {'img_loss': ((y - gt['img']) ** 2).mean()}
    if name == 'gradients_mse':
        g = torch_gradient(y, x)
        return {'gradients_loss': torch.mean((g - gt['gradients']).pow(2).sum(-1))}
    if name == 'laplace_mse':
        return {'laplace_loss': torch.mean((torch_laplace(y, x) - gt['laplace']) ** 2)}
    if name == 'sdf':
        g = torch_gradient(y, x)
        on = gt['sdf'] != -1
        sdf_c = torch.where(on, y, torch.zeros_like(y))
        inter = torch.where(on, torch.zeros_like(y), torch.exp(-1e2 * torch.abs(y)))
        normal = torch.where(on, 1 - F.cosine_similarity(g, gt['normals'], dim=-1)[..., None],
                             torch.zeros_like(g[..., :1]))
        gradc = torch.abs(g.norm(dim=-1) - 1)
        return {'sdf': torch.abs(sdf_c).mean() * 3e3, 'inter': inter.mean() * 1e2,
                'normal_constraint': normal.mean() * 1e2, 'grad_constraint': gradc.mean() * 5e1}
    raise KeyError(name)


def torch_param_grads(name, x, layers, gt, dtype='float64', **kw):
    """Flat theta-gradient of sum(loss.mean()) (training.py:75-96) through the torch restatement."""
    import torch
    dt = getattr(torch, dtype)
    params = []
    for W, b in layers:
        params += [torch.tensor(np.asarray(W), dtype=dt, requires_grad=True),
                   torch.tensor(np.asarray(b), dtype=dt, requires_grad=True)]
    xt = torch.tensor(np.asarray(x), dtype=dt, requires_grad=True)
    y = torch_forward(xt, params, **kw)
    gtt = {k: torch.tensor(np.asarray(v), dtype=dt) for k, v in gt.items()}
    terms = torch_loss_terms(name, y, xt, gtt)
    total = sum(v.mean() for v in terms.values())
    grads = torch.autograd.grad(total, params, allow_unused=True)
    grads = [torch.zeros_like(p) if g is None else g for g, p in zip(grads, params)]
    return np.concatenate([g.detach().numpy().reshape(-1) for g in grads]), float(total.detach())


# ----------------------------------------------------------------------------------------------------------
# per-step work: the device sampler's counter RNG and Adam + clip, restated
# ----------------------------------------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def _mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _rng64(seed, step, i):
    return _mix64((_mix64(seed ^ _mix64(step)) + i) & _M64)


def sample_sdf(pc, pn, k, seed, step):
    """dataio.PointCloud.__getitem__ (dataio.py:420-442) with the counter RNG of siren_sample_sdf
    (siren_amd/csrc/step_kernels.hpp): rows [0, k) = pc/pn[floor(r m / 2^64)], sdf 0; rows [k, 2k) = uniform
    2 u - 1 with u = (r >> 40) 2^-24, normals -1, sdf -1. Exact (integer arithmetic, fp32-exact floats)."""
    m = pc.shape[0]
    idx = np.array([(_rng64(seed, step, i) * m) >> 64 for i in range(k)], dtype=np.int64)
    u = np.array([[_rng64(seed, step, k + 3 * j + q) >> 40 for q in range(3)] for j in range(k)], dtype=np.float64)
    off = (2. * (u * 2. ** -24) - 1.).astype(np.float32)
    coords = np.concatenate([pc[idx], off], 0).astype(np.float32)
    normals = np.concatenate([pn[idx], -np.ones((k, 3), np.float32)], 0).astype(np.float32)
    sdf = np.concatenate([np.zeros((k, 1), np.float32), -np.ones((k, 1), np.float32)], 0)
    return coords, normals, sdf, idx


def adam_steps(p, grads, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, max_norm=None):
    """torch.optim.Adam (amsgrad off, no weight decay) after clip_grad_norm_ (training.py:17, 98-104), fp64, over a
    flat vector for a sequence of gradients; returns the final parameters."""
    p = np.array(p, np.float64)
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    for t, g in enumerate(grads, 1):
        g = np.array(g, np.float64)
        if max_norm:
            g = g * min(1., max_norm / (np.sqrt(np.sum(g * g)) + 1e-6))
        m = m + (1 - betas[0]) * (g - m)
        v = betas[1] * v + (1 - betas[1]) * g * g
        p = p - lr / (1 - betas[0] ** t) * m / (np.sqrt(v) / np.sqrt(1 - betas[1] ** t) + eps)
    return p
