"""The notebook API on the HIP kernels: Siren / SineLayer (explore_siren.ipynb cells 3 and 5) at hidden 256 —
outermost_linear True / False, first_omega_0 30 / 3000 — through Siren.forward's (output, coords) return and the
notebook's gradient / laplace (torch.autograd.grad with create_graph, the same op sequence as diff_operators.py),
against the reference notebook's own outputs (G8, tests/golden/make_golden.py). Needs an MI355X.

Tolerances, against the fp64 reference: model_out abs <= max(1e-4, 4 x the reference's own fp32
error); gradient / Laplacian abs <= 1e-4 * max(1, max|ref|) or 4 x the reference's fp32 error when larger (the
first_omega_0 = 3000 audio net: phases up to ~3000 rad); theta-grads abs <= 1e-4 * max|ref|.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = {'A': ((2, 256, 3, 1), dict(outermost_linear=True), 0),
         'B': ((1, 256, 3, 1), dict(outermost_linear=True, first_omega_0=3000, hidden_omega_0=30.), 1),
         'C': ((2, 256, 3, 3), dict(outermost_linear=False), 2)}


def nb_gradient(y, x):
    return torch.autograd.grad(y, [x], grad_outputs=torch.ones_like(y), create_graph=True)[0]


def nb_laplace(y, x):
    g = nb_gradient(y, x)
    div = 0.
    for i in range(g.shape[-1]):
        div += torch.autograd.grad(g[..., i], x, torch.ones_like(g[..., i]), create_graph=True)[0][..., i:i + 1]
    return div


def tol(fx, key, rel=1e-4):
    r64, r32 = fx[key + '_f64'], fx[key + '_f32']
    return max(rel * max(1., float(np.max(np.abs(r64)))), 4. * float(np.max(np.abs(r32 - r64))))


def siren(fx, tag, cuda, jet='auto'):
    from siren_amd.modules import Siren
    args, kw, _ = CASES[tag]
    s = Siren(*args, jet=jet, **kw)
    s.load_state_dict({k[len(tag) + 3:]: torch.tensor(v) for k, v in fx.items() if k.startswith(tag + '_w_')})
    return s.to(cuda)


@pytest.mark.parametrize('tag', ['A', 'B', 'C'])
@pytest.mark.parametrize('jet', [False, True])
def test_notebook_siren_forward_and_gradient_vs_reference(cuda, g8, tag, jet, monkeypatch):
    from siren_amd import _torch_path

    def boom(*a, **k):
        raise AssertionError('device-torch recompute used')
    monkeypatch.setattr(_torch_path, 'forward', boom)
    s = siren(g8, tag, cuda, jet)
    coords = torch.tensor(g8[tag + '_coords'], device=cuda)
    out, x = s(coords)
    assert x.requires_grad and x.is_leaf and x.shape == coords.shape and out.shape[:-1] == coords.shape[:-1]
    y64 = g8[tag + '_model_out_f64']
    assert np.max(np.abs(out.detach().cpu().numpy() - y64)) <= max(1e-4, tol(g8, tag + '_model_out'))
    g = nb_gradient(out, x)
    assert np.max(np.abs(g.detach().cpu().numpy() - g8[tag + '_gradient_f64'])) <= tol(g8, tag + '_gradient')


def test_notebook_siren_laplace_and_theta_grads_vs_reference(cuda, g8):
    """Case A: the notebook's laplace(gradient) op sequence (third-order nodes on the HIP kernels) and an image-mse
    training backward through Siren.forward."""
    s = siren(g8, 'A', cuda)
    coords = torch.tensor(g8['A_coords'], device=cuda)
    out, x = s(coords)
    lap = nb_laplace(out, x)
    assert np.max(np.abs(lap.detach().cpu().numpy() - g8['A_laplace_f64'])) <= tol(g8, 'A_laplace')
    s.zero_grad()
    out, _ = s(coords)
    loss = ((out - torch.sin(5 * coords[..., :1])) ** 2).mean()
    loss.backward()
    for k, p in s.named_parameters():
        ref = g8['A_image_mse_grad_' + k]
        assert np.max(np.abs(p.grad.cpu().numpy() - ref)) <= 1e-4 * np.max(np.abs(ref)), k
