"""Parity of the W4 jet kernel (siren_forward_laplace: y, grad and Laplacian in one forward-mode launch) and of
the fused diff_operators.laplace path against the reference's goldens and the fp64 oracle. Needs an MI355X.
Tolerances: y abs 1e-4; grad and Laplacian 1e-4 * max(1, max|ref|), against fp64 references.
"""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as O
from conftest import forbid_torch_path, weights_of

pytestmark = pytest.mark.gpu


def tol_rel(ref, rel=1e-4):
    return rel * max(1., float(np.max(np.abs(ref))))


def engine(d=2, L=3, o=1):
    from siren_amd.engine import SirenEngine
    return SirenEngine(d, 256, L, o)


def random_layers(d, L, o, seed=0, w=30.):
    rng = np.random.default_rng(seed)
    dims = [d] + [256] * (L + 1) + [o]
    layers = []
    for i, (fi, fo) in enumerate(zip(dims[:-1], dims[1:])):
        bound = 1. / fi if i == 0 else np.sqrt(6. / fi) / w
        layers.append((rng.uniform(-bound, bound, (fo, fi)).astype(np.float32),
                       (rng.uniform(-1, 1, fo) / np.sqrt(fi)).astype(np.float32)))
    return layers


def to_dev(a, dev):
    return torch.tensor(np.asarray(a, np.float32), device=dev)


@pytest.mark.parametrize('name', ['g1', 'g2'])
def test_w4_vs_reference_golden(cuda, name, request):
    """G1 (init weights) and G2 (300-step trained weights: |grad| ~ 1e2, |Laplacian| ~ 1e5)."""
    fx = request.getfixturevalue(name)
    g1 = request.getfixturevalue('g1')
    tag = name.upper()
    flat, _ = weights_of(fx)
    eng = engine()
    ws = eng.pack(to_dev(flat, cuda))
    y, gx, lap = eng.forward_laplace(ws, to_dev(g1['coords'][0], cuda), want_y=True, want_gx=True)
    ry, rg, rl = fx[tag + '_model_out_f64'][0], fx[tag + '_gradient_f64'][0], fx[tag + '_laplace_f64'][0]
    assert np.max(np.abs(y.cpu().numpy() - ry)) <= 1e-4
    assert np.max(np.abs(gx.cpu().numpy() - rg)) <= tol_rel(rg)
    assert np.max(np.abs(lap.cpu().numpy() - rl)) <= tol_rel(rl)


@pytest.mark.parametrize('n,d,L', [(1, 2, 3), (15, 2, 1), (17, 1, 2), (1000, 1, 3), (4097, 2, 4), (333, 2, 5)])
def test_w4_shapes_vs_oracle(cuda, n, d, L):
    layers = random_layers(d, L, 1, seed=n + 10 * L)
    eng = engine(d, L, 1)
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    x = np.random.default_rng(n).uniform(-1, 1, (n, d)).astype(np.float32)
    y, gx, lap = eng.forward_laplace(ws, to_dev(x, cuda), want_y=True, want_gx=True)
    ry, rg, rl = O.forward_laplace(x, layers)
    assert np.max(np.abs(y.cpu().numpy() - ry)) <= 1e-4
    assert np.max(np.abs(gx.cpu().numpy() - rg)) <= tol_rel(rg)
    assert np.max(np.abs(lap.cpu().numpy() - rl)) <= tol_rel(rl)
    _, lap_only = eng.forward_laplace(ws, to_dev(x, cuda))[1:]  # y / grad not requested
    assert torch.equal(lap_only, lap)


def test_w4_multi_output_sums_channels(cuda):
    """o > 1: laplace(y, x) = divergence(gradient(y, x)) sums the output channels (diff_operators.py:27-43)."""
    layers = random_layers(2, 2, 3, seed=5)
    eng = engine(2, 2, 3)
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    x = np.random.default_rng(5).uniform(-1, 1, (500, 2)).astype(np.float32)
    y, gx, lap = eng.forward_laplace(ws, to_dev(x, cuda), want_y=True, want_gx=True)
    rl = 0.
    rg = 0.
    for j in range(3):
        lj = [(W, b) for W, b in layers[:-1]] + [(layers[-1][0][j:j + 1], layers[-1][1][j:j + 1])]
        _, g_j, l_j = O.forward_laplace(x, lj)
        rl, rg = rl + l_j, rg + g_j
    assert np.max(np.abs(y.cpu().numpy() - O.forward(x, layers))) <= 1e-4
    assert np.max(np.abs(gx.cpu().numpy() - rg)) <= tol_rel(rg)
    assert np.max(np.abs(lap.cpu().numpy() - rl)) <= tol_rel(rl)


def test_w4_full_grid_properties(cuda):
    """BASELINE config 5 size: 512^2 get_mgrid grid. Subset vs oracle, bitwise determinism, agreement with
    the W1 gradient."""
    from siren_amd import dataio
    layers = random_layers(2, 3, 1, seed=9)
    eng = engine()
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    x = dataio.get_mgrid(512).to(cuda)
    y, gx, lap = eng.forward_laplace(ws, x, want_y=True, want_gx=True)
    y2, gx2, lap2 = eng.forward_laplace(ws, x, want_y=True, want_gx=True)
    assert torch.equal(lap, lap2) and torch.equal(gx, gx2) and torch.equal(y, y2)
    y1, g1 = eng.forward_grad(ws, x)
    assert torch.allclose(y, y1, rtol=0, atol=2e-6)
    assert torch.allclose(gx, g1, rtol=0, atol=1e-5 * float(g1.abs().max()))
    idx = torch.randperm(x.shape[0], generator=torch.Generator().manual_seed(0))[:1000]
    _, _, rl = O.forward_laplace(x[idx].cpu().numpy(), layers)
    assert np.max(np.abs(lap[idx].cpu().numpy() - rl)) <= tol_rel(rl)


def test_diff_operators_laplace_takes_the_fused_path(cuda, g2, monkeypatch):
    from siren_amd import diff_operators as D
    from siren_amd.engine import SirenEngine
    from siren_amd.modules import SingleBVPNet
    m = SingleBVPNet(verbose=False).to(cuda)
    m.load_state_dict({k[2:]: torch.tensor(v) for k, v in g2.items() if k.startswith('w_')})
    calls = []
    real, real_s = SirenEngine.forward_laplace, SirenEngine.forward_laplace_store  # (training: the split form)
    monkeypatch.setattr(SirenEngine, 'forward_laplace', lambda self, *a, **k: calls.append(1) or real(self, *a, **k))
    monkeypatch.setattr(SirenEngine, 'forward_laplace_store',
                        lambda self, *a, **k: calls.append(2) or real_s(self, *a, **k))
    coords = (torch.rand(1, 3000, 2, generator=torch.Generator().manual_seed(3)) * 2 - 1).to(cuda)
    out = m({'coords': coords})
    lap = D.laplace(out['model_out'], out['model_in'])
    assert calls and lap.shape == (1, 3000, 1)
    ref = D.divergence(D.gradient(out['model_out'], out['model_in']), out['model_in'])  # generic autograd path
    r = ref.detach().cpu().numpy()
    assert np.max(np.abs(lap.detach().cpu().numpy() - r)) <= tol_rel(r)


def _laplace_vjp_ref(x, layers, glap):
    """fp64 torch restatement: d/d(x, theta) of sum glap * laplace(y, x) (diff_operators.py:27-36)."""
    xt = torch.tensor(x, dtype=torch.float64, requires_grad=True)
    params = [torch.tensor(np.asarray(t), dtype=torch.float64, requires_grad=True) for W, b in layers for t in (W, b)]
    lap = O.torch_laplace(O.torch_forward(xt, params), xt)
    gs = torch.autograd.grad(lap, [xt] + params, torch.tensor(glap, dtype=torch.float64), allow_unused=True)
    gs = [torch.zeros_like(t) if g is None else g for g, t in zip(gs, [xt] + params)]  # b_out: no Laplacian term
    return gs[0].numpy(), torch.cat([g.reshape(-1) for g in gs[1:]]).numpy()


@pytest.mark.parametrize('n,d,L,o', [(1, 2, 3, 1), (50, 1, 2, 1), (777, 2, 3, 1), (2000, 2, 1, 2), (300, 2, 5, 1)])
def test_w4s_laplace_backward_vs_oracle(cuda, n, d, L, o):
    layers = random_layers(d, L, o, seed=3 * n + L)
    eng = engine(d, L, o)
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n)
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    glap = (rng.normal(size=(n, 1)) / n).astype(np.float32)
    gx, gp = eng.laplace_backward(ws, to_dev(x, cuda), to_dev(glap, cuda))
    rgx, rgp = _laplace_vjp_ref(x, layers, glap)
    assert np.max(np.abs(gp.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))
    assert np.max(np.abs(gx.cpu().numpy() - rgx)) <= 1e-4 * max(1e-6, np.max(np.abs(rgx)))


def test_w4s_deterministic_and_linear(cuda):
    from siren_amd import dataio
    layers = random_layers(2, 3, 1, seed=21)
    eng = engine()
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    x = dataio.get_mgrid(512).to(cuda)
    glap = torch.randn(x.shape[0], 1, device=cuda) / x.shape[0]
    a = eng.laplace_backward(ws, x, glap)
    b = eng.laplace_backward(ws, x, glap)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    c = eng.laplace_backward(ws, x, 3. * glap)
    assert torch.allclose(c[1], 3. * a[1], rtol=0, atol=1e-5 * float(a[1].abs().max()))


def test_laplace_mse_step_runs_on_hip_kernels(cuda, g1, monkeypatch):
    """laplace_mse training through the drop-in API: forward = W4, backward = W4s; no device-torch recompute."""
    from siren_amd import loss_functions as LF
    from siren_amd.modules import SingleBVPNet

    forbid_torch_path(monkeypatch)
    m = SingleBVPNet(verbose=False).to(cuda)
    m.load_state_dict({k[2:]: torch.tensor(v) for k, v in g1.items() if k.startswith('w_')})
    out = m({'coords': to_dev(g1['coords'], cuda)})
    loss = LF.laplace_mse(out, {'laplace': to_dev(g1['gt_laplace'], cuda)})['laplace_loss']
    loss.backward()
    for k, p in m.named_parameters():
        ref = g1['G1_laplace_mse_grad_' + k]
        assert np.max(np.abs(p.grad.cpu().numpy() - ref)) <= 1e-4 * np.max(np.abs(ref)) + 1e-12, k


@pytest.mark.parametrize('n,d,L', [(1, 2, 3), (4097, 2, 3), (1000, 1, 2), (333, 2, 5)])
def test_split_laplace_forward_backward_matches(cuda, n, d, L):
    """Split W4 / W4s (forward jet keeps its stores, reverse-only backward) == the single-launch kernels. The split's
    forward is the interleaved W4 kernel (w1_kernel MODE_JETS) and the single launch jet_store_kernel: same arithmetic
    per element, different GEMM accumulation order, so they agree to fp32 rounding (both are pinned against the fp64
    goldens by the tests above)."""
    from siren_amd.engine import SirenEngine
    rng = np.random.default_rng(n + L)
    dims = [d] + [256] * (L + 1) + [1]
    layers = []
    for i, (fi, fo) in enumerate(zip(dims[:-1], dims[1:])):
        bound = 1. / fi if i == 0 else np.sqrt(6. / fi) / 30.
        layers.append((rng.uniform(-bound, bound, (fo, fi)).astype(np.float32),
                       (rng.uniform(-1, 1, fo) / np.sqrt(fi)).astype(np.float32)))
    eng = SirenEngine(d, 256, L, 1)
    ws = eng.pack(torch.tensor(O.flatten(layers), device=cuda))
    x = torch.tensor(rng.uniform(-1, 1, (n, d)).astype(np.float32), device=cuda)
    glap = torch.tensor(rng.normal(size=(n, 1)).astype(np.float32), device=cuda)
    lap_s, tws = eng.forward_laplace_store(ws, x)
    _, _, lap_r = eng.forward_laplace(ws, x)
    assert float((lap_s - lap_r).abs().max()) <= 1e-5 * max(1., float(lap_r.abs().max()))
    gx_s, gp_s = eng.laplace_backward_stored(ws, x, glap, tws)
    gx_r, gp_r = eng.laplace_backward(ws, x, glap)
    assert float((gx_s - gx_r).abs().max()) <= 1e-5 * max(1., float(gx_r.abs().max()))
    assert float((gp_s - gp_r).abs().max()) <= 1e-5 * float(gp_r.abs().max())


def test_laplace_mse_one_forward_sweep(cuda, g1, monkeypatch):
    """From the second step on (the module's output went to diff_operators.laplace: JetState.laplace) the module's
    forward IS the W4 jet sweep (y from the same launch, its Laplacian and kept stores handed to fused_laplace): no
    stored W1 forward, one jet forward, one reverse-only W4s backward — and the step still matches the reference's
    fp64 laplace_mse theta-grads (G1), its Laplacian and its model output."""
    from siren_amd import loss_functions as LF
    from siren_amd.engine import SirenEngine
    from siren_amd.modules import SingleBVPNet
    calls = {'fwd_store': 0, 'lap_store': 0, 'lap_bwd_stored': 0}
    orig = {k: getattr(SirenEngine, k) for k in ('forward_store', 'forward_laplace_store', 'laplace_backward_stored')}

    def wrap(name, key):
        def f(self, *a, **k):
            calls[key] += 1
            return orig[name](self, *a, **k)
        return f
    monkeypatch.setattr(SirenEngine, 'forward_store', wrap('forward_store', 'fwd_store'))
    monkeypatch.setattr(SirenEngine, 'forward_laplace_store', wrap('forward_laplace_store', 'lap_store'))
    monkeypatch.setattr(SirenEngine, 'laplace_backward_stored', wrap('laplace_backward_stored', 'lap_bwd_stored'))
    m = SingleBVPNet(verbose=False).to(cuda)
    m.load_state_dict({k[2:]: torch.tensor(v) for k, v in g1.items() if k.startswith('w_')})
    gt = {'laplace': to_dev(g1['gt_laplace'], cuda)}
    for step in range(3):
        for k in calls:
            calls[k] = 0
        m.zero_grad()
        out = m({'coords': to_dev(g1['coords'], cuda)})
        losses = LF.laplace_mse(out, gt)
        losses['laplace_loss'].backward()
        if step >= 1:
            assert calls == {'fwd_store': 0, 'lap_store': 1, 'lap_bwd_stored': 1}, (step, calls)
            for k, p in m.named_parameters():
                ref = g1['G1_laplace_mse_grad_' + k]
                assert np.max(np.abs(p.grad.cpu().numpy() - ref)) <= 1e-4 * np.max(np.abs(ref)) + 1e-12, k
            y = out['model_out'].detach().cpu().numpy()
            assert np.max(np.abs(y - g1['G1_model_out_f64'])) <= 1e-4
    # a no_grad evaluation after laplace training keeps the plain forward (no jet sweep)
    jets = {'n': 0}
    orig_fl = SirenEngine.forward_laplace

    def fl(self, *a, **k):
        jets['n'] += 1
        return orig_fl(self, *a, **k)
    monkeypatch.setattr(SirenEngine, 'forward_laplace', fl)
    for k in calls:
        calls[k] = 0
    with torch.no_grad():
        y = m({'coords': to_dev(g1['coords'], cuda)})['model_out'].cpu().numpy()
    assert jets['n'] == 0 and calls['lap_store'] == 0
    assert np.max(np.abs(y - g1['G1_model_out_f64'])) <= 1e-4
