"""The losses of the reference's gradient-composition and inpainting scripts (loss_functions.py:22-56, 92-101) against
the reference's own outputs (G13, tests/golden/make_golden.py make_g13): gradients_color_mse on an RGB network and the
TV / FH inpainting priors, which call the model a second time per step on N/2 random points and train through its
gradient (TV, second order) or its Hessian (FH, third order).

CPU: siren_amd.loss_functions' restatements on the oracle's fp64 torch network (oracle/siren_oracle.py) reproduce the
reference's loss terms, random draws and fp64 theta-grads. GPU: the drop-in SingleBVPNet trains through them on the HIP
kernels with every device-torch recompute forbidden, three steps (jet mode and the per-call speculation of JetState
switch on from the second and third), each against the fp64 golden."""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as O
from conftest import forbid_torch_path, load_golden

CASES = [('C3', 'gradients_color_mse', 3), ('T1', 'image_mse_TV_prior', 1), ('T3', 'image_mse_TV_prior', 3),
         ('F1', 'image_mse_FH_prior', 1), ('F3', 'image_mse_FH_prior', 3)]
KEYS = ['net.net.%d.0.%s' % (i, k) for i in range(5) for k in ('weight', 'bias')]


@pytest.fixture(scope='module')
def g13():
    return load_golden('g13')


def _call(L, lname, tag, fx, manifest, model, out, dev, dtype):
    gt = {'img': torch.tensor(fx[tag + '_gt_img'], dtype=dtype, device=dev),
          'gradients': torch.tensor(fx[tag + '_gt_gradients'], dtype=dtype, device=dev)}
    mask = fx.get(tag + '_mask')
    mask = None if mask is None else torch.tensor(mask, dtype=dtype, device=dev)
    torch.manual_seed(manifest['G13_%s_rand_seed' % tag])  # the draw of the reference's run (global CPU generator)
    if lname == 'gradients_color_mse':
        return L.gradients_color_mse(out, gt)
    return getattr(L, lname)(mask, manifest['G13_%s_k1' % tag], model, out, gt)


def _ref_grads(fx, tag, dt):
    return {k: fx['%s_grad_%s_%s' % (tag, dt, k)] for k in KEYS}


@pytest.mark.parametrize('tag,lname,o', CASES)
def test_restated_losses_vs_reference_fp64(g13, manifest, tag, lname, o):
    """The restatements (siren_amd.loss_functions) on the oracle's fp64 CPU network: loss terms, the priors' random
    coordinates and theta-grads as the reference computes them."""
    from siren_amd import loss_functions as L
    layers = O.layers_from_state(g13, prefix=tag + '_w_')
    params = [torch.tensor(t, dtype=torch.float64, requires_grad=True) for W, b in layers for t in (W, b)]
    drawn = []

    def model(inp):
        c = inp['coords'].to(torch.float64).clone().detach().requires_grad_(True)
        drawn.append(c.detach().clone())
        return {'model_in': c, 'model_out': O.torch_forward(c, params)}
    out = model({'coords': torch.tensor(g13['coords'])})
    drawn.clear()
    ld = _call(L, lname, tag, g13, manifest, model, out, 'cpu', torch.float64)
    if lname != 'gradients_color_mse':
        assert len(drawn) == 1 and np.array_equal(drawn[0].numpy(), g13[tag + '_rand_coords'].astype(np.float64))
    for k, v in ld.items():
        ref = manifest['G13_%s_%s_f64' % (tag, k)]
        assert abs(float(v.detach()) - ref) <= 1e-9 * max(1., abs(ref)), (k, float(v.detach()), ref)
    total = sum(v.mean() for v in ld.values())
    grads = torch.autograd.grad(total, params, allow_unused=True)
    for k, g, p in zip(KEYS, grads, params):
        ref = g13['%s_grad_f64_%s' % (tag, k)]
        got = np.zeros(tuple(p.shape)) if g is None else g.numpy()
        assert np.max(np.abs(got - ref)) <= 1e-6 * max(np.max(np.abs(ref)), 1e-30), k


@pytest.mark.gpu
@pytest.mark.parametrize('tag,lname,o', CASES)
def test_losses_train_on_kernels_vs_reference(cuda, g13, manifest, tag, lname, o, monkeypatch):
    """Three training steps through the drop-in module with every _torch_path function forbidden; each step's loss
    terms and theta-grads against the reference's fp64 values. The bar is 1e-4 of max|ref| or twice the reference's
    own fp32-vs-fp64 difference where that is larger (the FH prior's Hessian norms pass through the reference's fp32
    hessian buffer, diff_operators.py:12, in its fp64 run too)."""
    from siren_amd import loss_functions as L
    from siren_amd.modules import SingleBVPNet
    forbid_torch_path(monkeypatch)
    m = SingleBVPNet(out_features=o, verbose=False).to(cuda)
    m.load_state_dict({k[len(tag) + 3:]: torch.tensor(v) for k, v in g13.items() if k.startswith(tag + '_w_')})
    ref64, ref32 = _ref_grads(g13, tag, 'f64'), _ref_grads(g13, tag, 'f32')
    coords = torch.tensor(g13['coords'], device=cuda)
    for step in range(3):
        m.zero_grad()
        out = m({'coords': coords})
        ld = _call(L, lname, tag, g13, manifest, m, out, cuda, torch.float32)
        for k, v in ld.items():
            r64, r32 = manifest['G13_%s_%s_f64' % (tag, k)], manifest['G13_%s_%s_f32' % (tag, k)]
            assert abs(float(v.detach()) - r64) <= max(1e-4 * max(1., abs(r64)), 2 * abs(r32 - r64)), (step, k)
        sum(v.mean() for v in ld.values()).backward()
        for k, p in m.named_parameters():
            r64, r32 = ref64[k], ref32[k]
            bar = max(1e-4 * np.max(np.abs(r64)), 2 * np.max(np.abs(r32 - r64))) + 1e-12
            got = np.zeros(tuple(p.shape)) if p.grad is None else p.grad.cpu().numpy()
            assert np.max(np.abs(got - r64)) <= bar, (step, k, np.max(np.abs(got - r64)), bar)
