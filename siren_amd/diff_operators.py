"""Coordinate differential operators with the reference's API (diff_operators.py:5-59).

They are thin autograd drivers, exactly like the reference's: the heavy lifting happens inside the
SirenFunction / SirenJacobian / SirenVJP nodes they differentiate through (siren_amd/autograd.py), so the
reference's own diff_operators module works unchanged against siren_amd models as well.
"""
import torch
from torch.autograd import grad


def gradient(y, x, grad_outputs=None):
    """dy/dx summed over y's channels (grad_outputs defaults to ones), differentiable (create_graph)."""
    if grad_outputs is None:
        grad_outputs = torch.ones_like(y)
    return torch.autograd.grad(y, [x], grad_outputs=grad_outputs, create_graph=True)[0]


def divergence(y, x):
    """sum_i d y_i / d x_i, one autograd call per input dimension (diff_operators.py:32-36)."""
    div = 0.
    for i in range(y.shape[-1]):
        div = div + grad(y[..., i], x, torch.ones_like(y[..., i]), create_graph=True)[0][..., i:i + 1]
    return div


def laplace(y, x):
    """divergence(gradient(y, x), x) (diff_operators.py:27-29). When y is a siren_amd SIREN's output of x, the whole
    Laplacian is ONE fused forward-mode kernel launch (W4, autograd.SirenLaplace) instead of d + 1 autograd
    sweeps; otherwise (or for networks the jet kernel does not cover) the reference's autograd recipe runs."""
    from .autograd import fused_laplace
    lap = fused_laplace(y, x)
    if lap is not None:
        return lap
    return divergence(gradient(y, x), x)


def jacobian(y, x):
    """(B, N, out, in) Jacobian and a NaN status flag (diff_operators.py:46-59)."""
    b, n = y.shape[:2]
    # the reference's buffer has the default dtype (diff_operators.py:49), so an fp64 graph is rounded to fp32 here
    jac = torch.zeros(b, n, y.shape[-1], x.shape[-1], device=y.device)
    for i in range(y.shape[-1]):
        y_flat = y[..., i].view(-1, 1)
        jac[:, :, i, :] = grad(y_flat, x, torch.ones_like(y_flat), create_graph=True)[0]
    status = -1 if torch.any(torch.isnan(jac)) else 0
    return jac, status


def hessian(y, x):
    """(B, N, out, in, in) Hessian and a NaN status flag (diff_operators.py:5-24)."""
    b, n = y.shape[:2]
    grad_y = torch.ones_like(y[..., 0])
    h = torch.zeros(b, n, y.shape[-1], x.shape[-1], x.shape[-1], device=y.device)  # default dtype, as :12
    for i in range(y.shape[-1]):
        dydx = grad(y[..., i], x, grad_y, create_graph=True)[0]
        for j in range(x.shape[-1]):
            h[..., i, j, :] = grad(dydx[..., j], x, grad_y, create_graph=True)[0][..., :]
    status = -1 if torch.any(torch.isnan(h)) else 0
    return h, status
