"""The loss consumers of the hot path (loss_functions.py:8-56, 80-109, 214-238), restated for the harness.

The reference's own loss_functions module runs unchanged against siren_amd models; these restatements exist so
the tests, smoke() and bench.py can run on the GPU box, where the reference is absent.
"""
import torch
import torch.nn.functional as F

from . import diff_operators


def image_mse(mask, model_output, gt):
    err = (model_output['model_out'] - gt['img']) ** 2
    return {'img_loss': (err if mask is None else mask * err).mean()}


def image_l1(mask, model_output, gt):
    err = torch.abs(model_output['model_out'] - gt['img'])
    return {'img_loss': (err if mask is None else mask * err).mean()}


def _rand_coords_like(model_in):
    """Uniform coordinates in [-1, 1) for the inpainting priors: (B, N // 2, d), drawn like the reference's
    2 * (torch.rand(...).cuda() - 0.5) (loss_functions.py:23-25, 40-42) — from the global CPU generator, then moved
    to the model's device — so a seeded run draws the reference's exact points (the arithmetic is exact in fp32)."""
    b, n, d = model_in.shape
    return (2 * (torch.rand((b, n // 2, d)) - 0.5)).to(device=model_in.device)


def image_mse_TV_prior(mask, k1, model, model_output, gt):
    """image_mse + k1 * mean |d model / dx| at N/2 random points (loss_functions.py:22-36): the prior is a second
    model call per step, and its gradient node's backward (the second-order W3 sweep) trains through it."""
    rand_output = model({'coords': _rand_coords_like(model_output['model_in'])})
    err = (model_output['model_out'] - gt['img']) ** 2
    prior = torch.abs(diff_operators.gradient(rand_output['model_out'], rand_output['model_in'])).mean()
    return {'img_loss': (err if mask is None else mask * err).mean(), 'prior_loss': k1 * prior}


def image_mse_FH_prior(mask, k1, model, model_output, gt):
    """image_mse + k1 * mean |Hessian|_F at N/2 random points (loss_functions.py:39-56): diff_operators.hessian of the
    second model call, so the prior trains through a third derivative (the shared Hessian node's backward)."""
    rand_output = model({'coords': _rand_coords_like(model_output['model_in'])})
    hes, _ = diff_operators.hessian(rand_output['model_out'], rand_output['model_in'])
    hes = hes.view(*hes.shape[0:2], -1)
    hnorm = hes.norm(dim=-1, keepdim=True)
    err = (model_output['model_out'] - gt['img']) ** 2
    return {'img_loss': (err if mask is None else mask * err).mean(), 'prior_loss': k1 * torch.abs(hnorm).mean()}


def function_mse(model_output, gt):
    return {'func_loss': ((model_output['model_out'] - gt['func']) ** 2).mean()}


def gradients_mse(model_output, gt):
    g = diff_operators.gradient(model_output['model_out'], model_output['model_in'])
    return {'gradients_loss': torch.mean((g - gt['gradients']).pow(2).sum(-1))}


def gradients_color_mse(model_output, gt):
    """Weighted per-channel gradient loss of an RGB network (loss_functions.py:92-101): one diff_operators.gradient
    per output channel (each a vjp node with a one-hot output weighting), concatenated to (B, N, 6)."""
    y, x = model_output['model_out'], model_output['model_in']
    g = torch.cat([diff_operators.gradient(y[..., c], x) for c in range(3)], dim=-1)
    weights = torch.tensor([1e1, 1e1, 1., 1., 1e1, 1e1], dtype=g.dtype, device=g.device)
    return {'gradients_loss': torch.mean((weights * (g[0:2] - gt['gradients']).pow(2)).sum(-1))}


def laplace_mse(model_output, gt):
    lap = diff_operators.laplace(model_output['model_out'], model_output['model_in'])
    return {'laplace_loss': torch.mean((lap - gt['laplace']) ** 2)}


def sdf(model_output, gt):
    gt_sdf, gt_normals = gt['sdf'], gt['normals']
    coords, pred = model_output['model_in'], model_output['model_out']
    g = diff_operators.gradient(pred, coords)
    on = gt_sdf != -1
    zeros = torch.zeros_like(pred)
    sdf_constraint = torch.where(on, pred, zeros)
    inter_constraint = torch.where(on, zeros, torch.exp(-1e2 * torch.abs(pred)))
    normal_constraint = torch.where(on, 1 - F.cosine_similarity(g, gt_normals, dim=-1)[..., None],
                                    torch.zeros_like(g[..., :1]))
    grad_constraint = torch.abs(g.norm(dim=-1) - 1)
    return {'sdf': torch.abs(sdf_constraint).mean() * 3e3,
            'inter': inter_constraint.mean() * 1e2,
            'normal_constraint': normal_constraint.mean() * 1e2,
            'grad_constraint': grad_constraint.mean() * 5e1}


def wave_pml(model_output, gt):
    """Wave-equation loss (loss_functions.py:112-136): Dirichlet + Neumann terms on the t = 0 set and the residual
    u_tt - c^2 (u_xx + u_yy) elsewhere. x = (t, x, y). The second derivatives are jacobian-of-jacobian: with
    siren_amd models both sweeps run on the HIP kernels (W1 vjp nodes, then the W3 kernel's vector-output form)."""
    from .diff_operators import jacobian
    sbv = gt['source_boundary_values']
    x, y = model_output['model_in'], model_output['model_out']
    slowness, mask = gt['squared_slowness'], gt['dirichlet_mask']
    batch_size = x.shape[1]
    du, _ = jacobian(y, x)
    dudt = du[..., 0]
    if torch.all(mask):
        diff_hom = torch.zeros(1, device=y.device, dtype=y.dtype)
    else:
        hess, _ = jacobian(du[..., 0, :], x)
        lap = hess[..., 1, 1, None] + hess[..., 2, 2, None]
        diff_hom = hess[..., 0, 0, None] - 1 / slowness * lap
    dirichlet = y[mask] - sbv[mask]
    neumann = dudt[mask]
    return {'dirichlet': torch.abs(dirichlet).sum() * batch_size / 1e1,
            'neumann': torch.abs(neumann).sum() * batch_size / 1e2,
            'diff_constraint_hom': torch.abs(diff_hom).sum()}


def helmholtz_pml(model_output, gt):
    """Helmholtz loss with a perfectly matched layer (loss_functions.py:139-211): complex field y = (re, im) per
    source, PML stretch factors ex, ey over the outer 0.5 of [-1, 1]^2, residual
    d/dx1 (ey/ex du/dx1) + d/dx2 (ex/ey du/dx2) + ex ey k^2 m u  (m = squared slowness), split into the source set
    and the rest; the 'pretrain' / full-waveform-inversion variants follow the reference's branches."""
    from .diff_operators import jacobian
    from .modules import compl_div, compl_mul
    sbv = gt['source_boundary_values']
    rec = gt.get('rec_boundary_values')
    k = gt['wavenumber'].float().to(model_output['model_out'].dtype)
    x, y = model_output['model_in'], model_output['model_out']
    slowness = gt['squared_slowness'].repeat(1, 1, y.shape[-1] // 2)
    batch_size = x.shape[1]
    fwi = False
    pred_slowness = None
    if 'pretrain' in gt:
        pred_slowness = y[:, :, -1] + 1.
        if torch.all(gt['pretrain'] == -1):
            fwi = True
            pred_slowness = torch.clamp(y[:, :, -1], min=-0.999) + 1.
            init = torch.stack((torch.ones_like(pred_slowness), torch.zeros_like(pred_slowness)), dim=-1)
            slowness = torch.stack((pred_slowness, torch.zeros_like(pred_slowness)), dim=-1)
            outer = (torch.abs(x[..., 0, None]) > 0.75) | (torch.abs(x[..., 1, None]) > 0.75)
            slowness = torch.where(outer, init, slowness)
        y = y[:, :, :-1]
    du, _ = jacobian(y, x)
    dudx1, dudx2 = du[..., 0], du[..., 1]
    a0, lpml = 5.0, 0.5
    d_w = -torch.clamp(x[..., 0] + (1.0 - lpml), max=0)
    d_e = torch.clamp(x[..., 0] - (1.0 - lpml), min=0)
    d_s = -torch.clamp(x[..., 1] + (1.0 - lpml), max=0)
    d_n = torch.clamp(x[..., 1] - (1.0 - lpml), min=0)
    sx = k * a0 * ((d_w / lpml) ** 2 + (d_e / lpml) ** 2)[..., None]
    sy = k * a0 * ((d_n / lpml) ** 2 + (d_s / lpml) ** 2)[..., None]
    ex = torch.cat((torch.ones_like(sx), -sx / k), dim=-1)
    ey = torch.cat((torch.ones_like(sy), -sy / k), dim=-1)
    reps = dudx1.shape[-1] // 2
    A = compl_div(ey, ex).repeat(1, 1, reps)
    B = compl_div(ex, ey).repeat(1, 1, reps)
    C = compl_mul(ex, ey).repeat(1, 1, reps)
    a, _ = jacobian(compl_mul(A, dudx1), x)
    b, _ = jacobian(compl_mul(B, dudx2), x)
    c = compl_mul(compl_mul(C, slowness), k ** 2 * y)
    diff_hom = a[..., 0] + b[..., 1] + c
    on = torch.where(sbv != 0., diff_hom - sbv, torch.zeros_like(diff_hom))
    off = torch.where(sbv == 0., diff_hom, torch.zeros_like(diff_hom))
    if fwi:
        data_term = torch.where(rec != 0, y - rec, torch.zeros_like(y))
    elif pred_slowness is not None:
        data_term = pred_slowness - slowness[..., 0]
    else:
        data_term = torch.zeros(1, device=y.device, dtype=y.dtype)
    return {'diff_constraint_on': torch.abs(on).sum() * batch_size / 1e3,
            'diff_constraint_off': torch.abs(off).sum(),
            'data_term': torch.abs(data_term).sum() * batch_size / 1}
