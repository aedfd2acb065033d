"""Device-side torch restatement of the SIREN op sequence, used ONLY for the higher-order adjoints that have no
HIP kernel yet: third derivatives (the backward of a Hessian-vector product node built by an unfused divergence or
the PML losses), theta-gradients under create_graph, and second derivatives of hidden-512 networks.

It runs on the same ROCm device as the kernels (never on the CPU) and re-records the reference's op order
(modules.py:23-24 matmul + bias, :34 sin(w z)) so autograd can differentiate it to any order. The first-order
path (W0, W1, W2) never touches this module.
"""
import torch


def unflatten(cfg, flat):
    d, H, L, o = cfg.d_in, cfg.hidden, cfg.n_hidden, cfg.d_out
    dims = [d] + [H] * (L + 1) + [o]
    out, off = [], 0
    for fi, fo in zip(dims[:-1], dims[1:]):
        W = flat[off:off + fo * fi].view(fo, fi)
        off += fo * fi
        b = flat[off:off + fo]
        off += fo
        out.append((W, b))
    return out


def forward(cfg, x, flat):
    layers = unflatten(cfg, flat)
    a = x
    for li, (W, b) in enumerate(layers):
        z = a.matmul(W.t()) + b
        last = li == len(layers) - 1
        if not (last and cfg.outermost_linear):
            z = torch.sin((cfg.omega_first if li == 0 else cfg.omega_hidden) * z)
        a = z
    return a


def _grads(outputs, inputs, grad_outputs, create_graph):
    live = [t for t in inputs if t is not None and t.requires_grad]
    got = iter(torch.autograd.grad(outputs, live, grad_outputs, create_graph=create_graph, allow_unused=True))
    res = []
    for t in inputs:
        if t is not None and t.requires_grad:
            g = next(got)
            res.append(torch.zeros_like(t) if g is None else g)
        else:
            res.append(None)
    return res


def vjp_params(cfg, x, flat, gy, create_graph):
    with torch.enable_grad():
        y = forward(cfg, x, flat)
        return _grads(y, [flat], gy, create_graph)[0]


def jacobian_vjp(cfg, x, flat, gJ, create_graph):
    """d/d(x, theta) of <gJ, dPhi/dx> (d_out == 1)."""
    with torch.enable_grad():
        y = forward(cfg, x, flat)
        J = torch.autograd.grad(y, x, torch.ones_like(y), create_graph=True)[0]
        gx, gp = _grads(J, [x, flat], gJ, create_graph)
    return gx, gp


def vjp_vjp(cfg, x, flat, gy, ggx, create_graph):
    """d/d(x, theta, gy) of <ggx, J^T gy>."""
    with torch.enable_grad():
        gyr = gy if gy.requires_grad else gy.detach().requires_grad_(True)
        y = forward(cfg, x, flat)
        gx = torch.autograd.grad(y, x, gyr, create_graph=True)[0]
        rx, rp, rgy = _grads(gx, [x, flat, gyr], ggx, create_graph)
    if not gy.requires_grad:
        rgy = None
    return rx, rp, rgy


def hvp_vjp(cfg, x, flat, v, g, create_graph, u=None):
    """d/d(x, theta, v, u) of <g, d/dx <v, J(x)^T u>> (u (n, d_out), None = ones)."""
    with torch.enable_grad():
        vr = v if v.requires_grad else v.detach().requires_grad_(True)
        ur = None
        if u is not None:
            ur = u if u.requires_grad else u.detach().requires_grad_(True)
        y = forward(cfg, x, flat)
        J = torch.autograd.grad(y, x, torch.ones_like(y) if ur is None else ur, create_graph=True)[0]
        hv = torch.autograd.grad(J, x, vr, create_graph=True)[0]
        rx, rp, rv, ru = _grads(hv, [x, flat, vr, ur], g, create_graph)
    if not v.requires_grad:
        rv = None
    if u is None or not u.requires_grad:
        ru = None
    return rx, rp, rv, ru


def hessian_vjp(cfg, x, flat, G, create_graph, u=None):
    """d/d(x, theta, u) of <G, Hm>, Hm[c, :, i] = sum_j u_j H_j(x_c) e_i (u (n, d_out), None = ones)."""
    with torch.enable_grad():
        ur = None
        if u is not None:
            ur = u if u.requires_grad else u.detach().requires_grad_(True)
        y = forward(cfg, x, flat)
        J = torch.autograd.grad(y, x, torch.ones_like(y) if ur is None else ur, create_graph=True)[0]
        S = 0.
        for i in range(x.shape[-1]):
            e = torch.zeros_like(J)
            e[:, i] = 1.
            S = S + (torch.autograd.grad(J, x, e, create_graph=True)[0] * G[:, :, i]).sum()
        rx, rp, ru = _grads(S, [x, flat, ur], None, create_graph)
    if u is None or not u.requires_grad:
        ru = None
    return rx, rp, ru


def laplacian(cfg, x, flat):
    """sum_j sum_i d2 Phi_j / dx_i2 as a differentiable graph (diff_operators.laplace's op sequence)."""
    y = forward(cfg, x, flat)
    g = torch.autograd.grad(y, x, torch.ones_like(y), create_graph=True)[0]
    lap = 0.
    for i in range(x.shape[-1]):
        lap = lap + torch.autograd.grad(g[:, i], x, torch.ones_like(g[:, i]), create_graph=True)[0][:, i:i + 1]
    return lap


def laplace_vjp(cfg, x, flat, glap, create_graph):
    """d/d(x, theta) of <glap, Laplacian(x; theta)> (the backward of the fused Laplacian node)."""
    with torch.enable_grad():
        lap = laplacian(cfg, x, flat)
        gx, gp = _grads(lap, [x, flat], glap, create_graph)
    return gx, gp
