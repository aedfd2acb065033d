"""The loss consumers of the hot path (loss_functions.py:8-12, 80-109, 214-238), restated for the harness.

The reference's own loss_functions module runs unchanged against siren_amd models; these restatements exist so
the tests, smoke() and bench.py can run on the GPU box, where the reference is absent.
"""
import torch
import torch.nn.functional as F

from . import diff_operators


def image_mse(mask, model_output, gt):
    err = (model_output['model_out'] - gt['img']) ** 2
    return {'img_loss': (err if mask is None else mask * err).mean()}


def function_mse(model_output, gt):
    return {'func_loss': ((model_output['model_out'] - gt['func']) ** 2).mean()}


def gradients_mse(model_output, gt):
    g = diff_operators.gradient(model_output['model_out'], model_output['model_in'])
    return {'gradients_loss': torch.mean((g - gt['gradients']).pow(2).sum(-1))}


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
