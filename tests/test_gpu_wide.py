"""Parity of the hidden-512 kernels (wide_kernel.hpp + the h = 512 wgrad/small kernels) against the reference's
G4 golden vectors (SingleBVPNet(in 3, out 3, hidden 512, 3 hidden layers), BASELINE config 4) and the fp64
oracle. Needs an MI355X. Tolerances as test_gpu_parity.py (1e-4 abs / relative to max|ref|).
"""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as O
from conftest import forbid_torch_path, weights_of

pytestmark = pytest.mark.gpu

H = 512


def tol_rel(ref, rel=1e-4):
    return rel * max(1., float(np.max(np.abs(ref))))


def wide_engine(d=3, L=3, o=3, w0=30., w=30., lin=True):
    from siren_amd.engine import SirenEngine
    return SirenEngine(d, H, L, o, w0, w, lin)


def random_layers(d, L, o, seed=0, w=30.):
    rng = np.random.default_rng(seed)
    dims = [d] + [H] * (L + 1) + [o]
    layers = []
    for i, (fi, fo) in enumerate(zip(dims[:-1], dims[1:])):
        bound = 1. / fi if i == 0 else np.sqrt(6. / fi) / w
        layers.append((rng.uniform(-bound, bound, (fo, fi)).astype(np.float32),
                       (rng.uniform(-1, 1, fo) / np.sqrt(fi)).astype(np.float32)))
    return layers


def to_dev(a, dev):
    return torch.tensor(np.asarray(a, np.float32), device=dev)


def test_g4_forward_gradient_vs_reference_golden(cuda, g4):
    flat, _ = weights_of(g4)
    eng = wide_engine()
    ws = eng.pack(to_dev(flat, cuda))
    x = to_dev(g4['coords'][0], cuda)
    y0 = eng.forward(ws, x).cpu().numpy()
    y1, gx = eng.forward_grad(ws, x)
    ry, rg = g4['G4_model_out_f64'][0], g4['G4_gradient_f64'][0]
    assert np.max(np.abs(y0 - ry)) <= 1e-4
    assert np.max(np.abs(y1.cpu().numpy() - ry)) <= 1e-4
    assert np.max(np.abs(gx.cpu().numpy() - rg)) <= tol_rel(rg)


def test_g4_image_mse_theta_grads_vs_reference_golden(cuda, g4):
    flat, layers = weights_of(g4)
    eng = wide_engine()
    ws = eng.pack(to_dev(flat, cuda))
    x = to_dev(g4['coords'][0], cuda)
    y = eng.forward(ws, x)
    gt = to_dev(g4['gt_img'][0], cuda)
    gy = 2. * (y - gt) / y.numel()
    gx, gp = eng.backward_params(ws, x, gy)
    keys = ['net.net.%d.0.%s' % (i, k) for i in range(5) for k in ('weight', 'bias')]
    ref = np.concatenate([g4['G4_image_mse_grad_' + k].reshape(-1) for k in keys])
    assert np.max(np.abs(gp.cpu().numpy() - ref)) <= 1e-4 * np.max(np.abs(ref))
    _, rgx = O.forward_grad(g4['coords'][0], layers, gy.cpu().numpy())
    assert np.max(np.abs(gx.cpu().numpy() - rgx)) <= 1e-4 * np.max(np.abs(rgx))


@pytest.mark.parametrize('n,d,L,o', [(1, 2, 1, 1), (100, 3, 2, 3), (5000, 2, 3, 1), (3000, 1, 5, 2)])
def test_wide_shapes_vs_oracle(cuda, n, d, L, o):
    layers = random_layers(d, L, o, seed=n + L)
    eng = wide_engine(d, L, o)
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n)
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    gy = rng.normal(size=(n, o)).astype(np.float32)
    xd, gyd = to_dev(x, cuda), to_dev(gy, cuda)
    y = eng.forward(ws, xd)
    y1, gx = eng.forward_grad(ws, xd, gyd)
    ry, rg = O.forward_grad(x, layers, gy)
    assert np.max(np.abs(y.cpu().numpy() - ry)) <= 1e-4
    assert np.max(np.abs(y1.cpu().numpy() - ry)) <= 1e-4
    assert np.max(np.abs(gx.cpu().numpy() - rg)) <= tol_rel(rg)
    gyn = gy / n
    gx2, gp = eng.backward_params(ws, xd, to_dev(gyn, cuda))
    xt = torch.tensor(x, dtype=torch.float64)
    params = [torch.tensor(np.asarray(t), dtype=torch.float64, requires_grad=True) for W, b in layers for t in (W, b)]
    yt = O.torch_forward(xt, params)
    ref = torch.cat([g.reshape(-1) for g in torch.autograd.grad(yt, params, torch.tensor(gyn, dtype=torch.float64))])
    ref = ref.numpy()
    assert np.max(np.abs(gp.cpu().numpy() - ref)) <= 1e-4 * np.max(np.abs(ref))
    assert np.max(np.abs(gx2.cpu().numpy() - rg / n)) <= tol_rel(rg / n)


def test_wide_final_sine_vs_oracle(cuda):
    """notebook Siren(outermost_linear=False) at hidden 512: sin on the output layer too."""
    layers = random_layers(2, 2, 1, seed=7)
    eng = wide_engine(2, 2, 1, lin=False)
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    x = np.random.default_rng(7).uniform(-1, 1, (777, 2)).astype(np.float32)
    y, gx = eng.forward_grad(ws, to_dev(x, cuda))
    ry, rg = O.forward_grad(x, layers, None, outermost_linear=False)
    assert np.max(np.abs(y.cpu().numpy() - ry)) <= 1e-4
    assert np.max(np.abs(gx.cpu().numpy() - rg)) <= tol_rel(rg)


def test_wide_deterministic_and_linear(cuda):
    layers = random_layers(3, 3, 3, seed=5)
    eng = wide_engine()
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    n = 1 << 17
    x = torch.rand(n, 3, device=cuda) * 2 - 1
    gy = torch.randn(n, 3, device=cuda)
    a = eng.backward_params(ws, x, gy)
    b = eng.backward_params(ws, x, gy)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    _, g1 = eng.forward_grad(ws, x, gy, want_y=False)
    _, g2 = eng.forward_grad(ws, x, 2. * gy, want_y=False)
    assert torch.allclose(g2, 2. * g1, rtol=0, atol=1e-6 * float(g1.abs().max()))
    # subset against the oracle
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(0))[:512]
    _, rg = O.forward_grad(x[idx].cpu().numpy(), layers, gy[idx].cpu().numpy())
    assert np.max(np.abs(g1[idx].cpu().numpy() - rg)) <= tol_rel(rg)


def test_module_image_fit_step_wide(cuda, g4):
    """Drop-in: SingleBVPNet(hidden_features=512) + loss_functions.image_mse + backward == reference golden."""
    from siren_amd.modules import SingleBVPNet
    from siren_amd import loss_functions as LF
    torch.manual_seed(0)
    m = SingleBVPNet(out_features=3, in_features=3, hidden_features=512, num_hidden_layers=3, verbose=False).to(cuda)
    out = m({'coords': to_dev(g4['coords'], cuda)})
    loss = LF.image_mse(None, out, {'img': to_dev(g4['gt_img'], cuda)})['img_loss']
    assert abs(float(loss.detach()) - 0.3987086920864164) <= 1e-5
    loss.backward()
    for name, p in m.named_parameters():
        ref = g4['G4_image_mse_grad_' + name]
        assert np.max(np.abs(p.grad.cpu().numpy() - ref)) <= 1e-4 * max(1e-6, np.max(np.abs(ref))) + 1e-9, name


@pytest.mark.parametrize('n,d,L,o', [(1, 3, 3, 3), (4097, 3, 3, 3), (700, 2, 1, 1), (333, 4, 5, 2), (130, 1, 2, 4),
                                     (2000, 3, 4, 3), (65536, 3, 3, 3)])
def test_wide_interleaved_split_bitwise_vs_serial(cuda, n, d, L, o):
    """The interleaved hidden-512 stored split (widei_kernel, default) against the serial one (wide_kernel,
    SIREN_FLAG_WIDE_SERIAL): the same arithmetic on another schedule, so y, the stored a_l tiles / cos scratch, gx and
    the theta-grads are bitwise equal."""
    from siren_amd.engine import SirenEngine
    layers = random_layers(d, L, o, seed=11 * n + L)
    eng, ser = wide_engine(d, L, o), SirenEngine(d, H, L, o, flags=16)
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n + 3)
    x = to_dev(rng.uniform(-1, 1, (n, d)), cuda)
    gy = to_dev(rng.normal(size=(n, o)), cuda)
    y_a, tws_a = eng.forward_store(ws, x)
    y_b, tws_b = ser.forward_store(ws, x)
    assert torch.equal(y_a, y_b)
    gx_a, gp_a = eng.backward_stored(ws, x, gy, tws_a)
    gx_b, gp_b = ser.backward_stored(ws, x, gy, tws_b)
    assert torch.equal(gx_a, gx_b) and torch.equal(gp_a, gp_b)
    assert torch.isfinite(gp_a).all()


@pytest.mark.parametrize('n,d,L,o', [(1, 3, 3, 3), (4097, 3, 3, 3), (700, 2, 1, 1), (333, 4, 5, 2)])
def test_wide_stored_forward_split_matches_recompute(cuda, n, d, L, o):
    """Hidden 512 stored-forward split (wide_kernel MODE_FWDS / MODE_REV) == the recompute pipeline; vs fp64."""
    layers = random_layers(d, L, o, seed=5 * n + L)
    eng = wide_engine(d, L, o)
    assert eng.stored_supported
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n + 1)
    x = to_dev(rng.uniform(-1, 1, (n, d)), cuda)
    gy = to_dev(rng.normal(size=(n, o)), cuda)
    y_s, tws = eng.forward_store(ws, x)
    gx_s, gp_s = eng.backward_stored(ws, x, gy, tws)
    y_r = eng.forward(ws, x)
    assert torch.equal(y_s, y_r)
    if eng.grad_supported:
        gx_r, gp_r = eng.backward_params(ws, x, gy)
        assert float((gx_s - gx_r).abs().max()) <= 1e-6 * max(1., float(gx_r.abs().max()))
        assert float((gp_s - gp_r).abs().max()) <= 1e-6 * float(gp_r.abs().max())
    xt = torch.tensor(x.cpu().numpy(), dtype=torch.float64, requires_grad=True)
    params = [torch.tensor(t, dtype=torch.float64, requires_grad=True) for W, b in layers for t in (W, b)]
    yt = O.torch_forward(xt, params)
    g = torch.autograd.grad(yt, [xt] + params, torch.tensor(gy.cpu().numpy(), dtype=torch.float64))
    rgp = torch.cat([t.reshape(-1) for t in g[1:]]).numpy()
    assert np.max(np.abs(gp_s.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))
    assert np.max(np.abs(gx_s.cpu().numpy() - g[0].numpy())) <= tol_rel(g[0].numpy())


# ---- second order at hidden 512 (wide_jet_kernel.hpp: two-stream jet) -------------------------------------------
def w3_ref(x, layers, v, u, gy):
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


@pytest.mark.parametrize('n,d,L,o,weighted,seeded', [(1, 2, 3, 1, False, False), (33, 2, 3, 1, False, True),
                                                      (1000, 3, 3, 3, True, True), (2053, 3, 1, 1, False, False),
                                                      (700, 1, 2, 2, True, False), (64, 4, 5, 4, True, True)])
def test_wide_second_order_vs_fp64(cuda, n, d, L, o, weighted, seeded):
    """H v, the mixed theta-gradient and J v at hidden 512 (siren_second_order_ex -> the two-stream jet kernel +
    MFMA wgrad over 2n columns + EDGE_J2) against fp64 autograd."""
    layers = random_layers(d, L, o, seed=5 * n + L)
    eng = wide_engine(d, L, o)
    assert eng.second_order_supported
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n + 3 * o)
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    v = rng.normal(size=(n, d)).astype(np.float32)
    u = rng.normal(size=(n, o)).astype(np.float32) if weighted else None
    gy = rng.normal(size=(n, o)).astype(np.float32) if seeded else None
    X, V = to_dev(x, cuda), to_dev(v, cuda)
    gx, gp, ydot = eng.second_order(ws, X, V, want_theta=True, gy=to_dev(gy, cuda) if seeded else None,
                                    u=to_dev(u, cuda) if weighted else None, want_ydot=True)
    gx2, none = eng.second_order(ws, X, V, want_theta=False, gy=to_dev(gy, cuda) if seeded else None,
                                 u=to_dev(u, cuda) if weighted else None)
    rgx, rgp, rjv = w3_ref(x, layers, v, u, gy)
    assert none is None and torch.equal(gx, gx2)
    assert np.max(np.abs(gx.cpu().numpy() - rgx)) <= tol_rel(rgx)
    assert np.max(np.abs(gp.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))
    assert np.max(np.abs(ydot.cpu().numpy() - rjv)) <= tol_rel(rjv)


@pytest.mark.parametrize('case', ['A', 'B'])
def test_g9_second_order_losses_at_hidden512_vs_reference(cuda, g9, manifest, case, monkeypatch):
    """gradients_mse (d2) and sdf (d3) training at hidden_features=512 through the drop-in API against the
    reference's fp64 theta-gradients (G9), with the device-torch second-order recompute forbidden; two passes (the
    second runs with jet mode switched on)."""
    from siren_amd.modules import SingleBVPNet
    from siren_amd import loss_functions as LF
    forbid_torch_path(monkeypatch)
    d = 2 if case == 'A' else 3
    m = SingleBVPNet(in_features=d, hidden_features=512, verbose=False).to(cuda)
    m.load_state_dict({k[len(case) + 3:]: torch.tensor(v) for k, v in g9.items() if k.startswith(case + '_w_')})
    coords = to_dev(g9[case + '_coords'], cuda)
    for _ in range(2):
        m.zero_grad()
        out = m({'coords': coords})
        if case == 'A':
            terms = LF.gradients_mse(out, {'gradients': to_dev(g9['A_gt_gradients'], cuda)})
            key = 'A_gradients_mse_grad_'
        else:
            terms = LF.sdf(out, {'sdf': to_dev(g9['B_gt_sdf'], cuda), 'normals': to_dev(g9['B_gt_normals'], cuda)})
            key = 'B_sdf_grad_'
            for k, t in terms.items():
                ref = manifest['G9_sdf_%s_f64' % k]
                assert abs(float(t.mean().detach()) - ref) <= 1e-4 * max(1., abs(ref)), k
        sum(t.mean() for t in terms.values()).backward()
        for k, p in m.named_parameters():
            ref = g9[key + k]
            assert np.max(np.abs(p.grad.cpu().numpy() - ref)) <= 1e-4 * np.max(np.abs(ref)) + 1e-12, k
