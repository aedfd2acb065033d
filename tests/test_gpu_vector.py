"""Vector outputs and the PML losses on the HIP kernels: the W3 kernel's output-weighted
form (siren_second_order_ex) against fp64 autograd, diff_operators.jacobian / hessian (diff_operators.py:5-24,
46-59) and the helmholtz_pml / wave_pml training gradients (loss_functions.py:112-211) against the reference's
G6 golden (tests/golden/make_golden.py). Needs an MI355X.

Tolerances as tests/test_gpu_parity.py: derivatives abs <= 1e-4 * max(1, max|ref|), theta-grads abs <= 1e-4 *
max|ref| against the fp64 reference (fp32 torch autograd of the same losses sits at 3e-7 / 4e-7 of max|ref|).
"""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as O
from conftest import forbid_torch_path, pml_case, pml_ref_grads

pytestmark = pytest.mark.gpu


def tol_rel(ref, rel=1e-4):
    return rel * max(1., float(np.max(np.abs(ref))))


def to_dev(a, dev):
    return torch.tensor(np.asarray(a, np.float32), device=dev)


def random_layers(d, L, o, seed=0, w=30.):
    rng = np.random.default_rng(seed)
    dims = [d] + [256] * (L + 1) + [o]
    layers = []
    for i, (fi, fo) in enumerate(zip(dims[:-1], dims[1:])):
        bound = 1. / fi if i == 0 else np.sqrt(6. / fi) / w
        layers.append((rng.uniform(-bound, bound, (fo, fi)).astype(np.float32),
                       (rng.uniform(-1, 1, fo) / np.sqrt(fi)).astype(np.float32)))
    return layers


def vector_w3_ref(x, layers, v, u, gy):
    """fp64 autograd: F = sum gy . y + <v, J^T u>; returns dF/dx, dF/dtheta, J v."""
    xt = torch.tensor(x, dtype=torch.float64, requires_grad=True)
    params = [torch.tensor(t, dtype=torch.float64, requires_grad=True) for W, b in layers for t in (W, b)]
    y = O.torch_forward(xt, params)
    ut = torch.ones_like(y) if u is None else torch.tensor(u, dtype=torch.float64)
    Ju = torch.autograd.grad(y, xt, ut, create_graph=True)[0]
    F = (Ju * torch.tensor(v, dtype=torch.float64)).sum()
    if gy is not None:
        F = F + (y * torch.tensor(gy, dtype=torch.float64)).sum()
    grads = torch.autograd.grad(F, [xt] + params, allow_unused=True, retain_graph=True)
    gp = torch.cat([(torch.zeros_like(p) if g is None else g).reshape(-1) for g, p in zip(grads[1:], params)])
    vt = torch.tensor(v, dtype=torch.float64)
    jv = torch.stack([(torch.autograd.grad(y[:, j].sum(), xt, retain_graph=True)[0] * vt).sum(-1)
                      for j in range(y.shape[1])], -1)
    return grads[0].numpy(), gp.detach().numpy(), jv.numpy()


@pytest.mark.parametrize('n,d,L,o,weighted,seeded', [(1, 2, 3, 2, True, False), (4097, 2, 3, 2, True, True),
                                                      (1000, 3, 3, 3, True, True), (333, 3, 2, 4, False, True),
                                                      (700, 4, 1, 2, True, False), (2048, 3, 3, 1, True, True)])
def test_w3_vector_output_vs_fp64(cuda, n, d, L, o, weighted, seeded):
    from siren_amd.engine import SirenEngine
    layers = random_layers(d, L, o, seed=11 * n + o)
    eng = SirenEngine(d, 256, L, o)
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n + o)
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    v = rng.normal(size=(n, d)).astype(np.float32)
    u = rng.normal(size=(n, o)).astype(np.float32) if weighted else None
    gy = rng.normal(size=(n, o)).astype(np.float32) if seeded else None
    X, V = to_dev(x, cuda), to_dev(v, cuda)
    U = to_dev(u, cuda) if weighted else None
    GY = to_dev(gy, cuda) if seeded else None
    gx, gp, ydot = eng.second_order(ws, X, V, want_theta=True, gy=GY, u=U, want_ydot=True)
    gx2, none = eng.second_order(ws, X, V, want_theta=False, gy=GY, u=U)
    rgx, rgp, rjv = vector_w3_ref(x, layers, v, u, gy)
    assert none is None and torch.equal(gx, gx2)
    assert np.max(np.abs(gx.cpu().numpy() - rgx)) <= tol_rel(rgx)
    assert np.max(np.abs(gp.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))
    assert np.max(np.abs(ydot.cpu().numpy() - rjv)) <= tol_rel(rjv)


def _model(case, cuda, d, o, jet='auto'):
    from siren_amd.modules import SingleBVPNet
    coords, gt, flat, layers = case
    m = SingleBVPNet(in_features=d, out_features=o, verbose=False, jet=jet).to(cuda)
    sd = {}
    for i, (W, b) in enumerate(layers):
        sd['net.net.%d.0.weight' % i] = torch.tensor(W)
        sd['net.net.%d.0.bias' % i] = torch.tensor(b)
    m.load_state_dict(sd)
    return m


def test_jacobian_hessian_vector_output_vs_reference(cuda, g6, monkeypatch):
    """d_out = 2 (a complex Helmholtz field): jacobian through W1 vjp nodes, hessian through the W3 kernel."""
    from siren_amd import diff_operators as D
    forbid_torch_path(monkeypatch)
    case = pml_case(g6, 'H')
    m = _model(case, cuda, 2, 2)
    out = m({'coords': to_dev(case[0], cuda)})
    y = out['model_out']
    assert np.max(np.abs(y.detach().cpu().numpy() - g6['H_model_out_f64'])) <= 1e-4
    jac, st = D.jacobian(y, out['model_in'])
    hes, st2 = D.hessian(y, out['model_in'])
    assert st == 0 and st2 == 0
    rj, rh = g6['H_jacobian_f64'], g6['H_hessian_f64']
    assert np.max(np.abs(jac.detach().cpu().numpy() - rj)) <= tol_rel(rj)
    assert np.max(np.abs(hes.detach().cpu().numpy() - rh)) <= tol_rel(rh)


@pytest.mark.parametrize('tag,d,o,jet', [('H', 2, 2, 'auto'), ('W', 3, 1, False), ('W', 3, 1, True)])
def test_pml_training_theta_grads_vs_reference(cuda, g6, manifest, monkeypatch, tag, d, o, jet):
    """helmholtz_pml / wave_pml training step: loss terms and theta-grads vs the reference's fp64 golden; the
    second-order sweeps run on W3 and the third-order ones on the mixed jet (every torch recompute is forbidden)."""
    from siren_amd import loss_functions as LF
    forbid_torch_path(monkeypatch)
    case = pml_case(g6, tag)
    coords, gt = case[0], case[1]
    m = _model(case, cuda, d, o, jet=jet)
    gtt = {k: (to_dev(v, cuda) if v.dtype != np.bool_ else torch.tensor(v, device=cuda)) for k, v in gt.items()}
    fn = LF.helmholtz_pml if tag == 'H' else LF.wave_pml
    name = 'helmholtz' if tag == 'H' else 'wave'
    for _ in range(2):  # the second pass runs with jet mode switched on ('auto')
        m.zero_grad()
        terms = fn(m({'coords': to_dev(coords, cuda)}), gtt)
        total = sum(v.mean() for v in terms.values())
        total.backward()
    for k, v in terms.items():
        ref = manifest['G6_%s_%s_f64' % (name, k)]
        assert abs(float(v.detach()) - ref) <= 1e-4 * max(1., abs(ref)), k
    gp = torch.cat([p.grad.reshape(-1) for p in m.parameters()]).cpu().numpy()
    ref = pml_ref_grads(g6, tag)
    assert np.max(np.abs(gp - ref)) <= 1e-4 * np.max(np.abs(ref))
