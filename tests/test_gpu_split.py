"""Parity of the split-bf16 W1 kernel (siren_forward_grad_split, w1x_kernel.hpp: bf16 hi/mid/lo pieces, six
products per K-step, fp32 accumulation) against the fp64 oracle and the reference's golden vectors, with the same
tolerances as the fp32 kernel and the extra requirement that its error stays at the fp32 kernel's
level (the split is an fp32-equivalent precision mode, not a reduced one). Needs an MI355X."""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as O
from conftest import forbid_torch_path, weights_of

pytestmark = pytest.mark.gpu


def tol_rel(ref, rel=1e-4):
    return rel * max(1., float(np.max(np.abs(ref))))


def engine(d=2):
    from siren_amd.engine import SirenEngine
    return SirenEngine(d, 256, 3, 1, 30., 30., True)


def random_layers(d, seed=0):
    rng = np.random.default_rng(seed)
    dims = [d] + [256] * 4 + [1]
    layers = []
    for i, (fi, fo) in enumerate(zip(dims[:-1], dims[1:])):
        bound = 1. / fi if i == 0 else np.sqrt(6. / fi) / 30.
        layers.append((rng.uniform(-bound, bound, (fo, fi)).astype(np.float32),
                       (rng.uniform(-1, 1, fo) / np.sqrt(fi)).astype(np.float32)))
    return layers


def to_dev(a, dev):
    return torch.tensor(np.asarray(a, np.float32), device=dev)


@pytest.mark.parametrize('name', ['g1', 'g2'])
def test_split_vs_reference_golden(cuda, name, request):
    fx = request.getfixturevalue(name)
    g1 = request.getfixturevalue('g1')
    tag = name.upper()
    flat, _ = weights_of(fx)
    eng = engine()
    fdev = to_dev(flat, cuda)
    ws, wsx = eng.pack(fdev), eng.pack_split(fdev)
    x = to_dev(g1['coords'][0], cuda)
    y, gx = eng.forward_grad_split(wsx, x)
    y32, gx32 = eng.forward_grad(ws, x)
    ry, rg = fx[tag + '_model_out_f64'][0], fx[tag + '_gradient_f64'][0]
    ey, eg = np.max(np.abs(y.cpu().numpy() - ry)), np.max(np.abs(gx.cpu().numpy() - rg))
    ey32, eg32 = np.max(np.abs(y32.cpu().numpy() - ry)), np.max(np.abs(gx32.cpu().numpy() - rg))
    print('%s split: |dy| %.2e |dg| %.2e   fp32 kernel: |dy| %.2e |dg| %.2e' % (name, ey, eg, ey32, eg32))
    assert ey <= 1e-4 and eg <= tol_rel(rg)
    # fp32-equivalent: within 2x of the fp32 kernel's own error (and of the reference's fp32 autograd, x4 margin)
    assert eg <= 2 * eg32 + 1e-6
    assert ey <= 2 * ey32 + 1e-7
    own = np.max(np.abs(fx[tag + '_gradient_f32'][0] - rg))
    assert eg <= 4 * own + 1e-6


@pytest.mark.parametrize('d', [2, 3])
@pytest.mark.parametrize('n', [1, 15, 63, 64, 65, 1000, 4097])
def test_split_ragged_sizes(cuda, n, d):
    layers = random_layers(d, seed=n + d)
    eng = engine(d)
    wsx = eng.pack_split(to_dev(O.flatten(layers), cuda))
    x = np.random.default_rng(n).uniform(-1, 1, (n, d)).astype(np.float32)
    y, gx = eng.forward_grad_split(wsx, to_dev(x, cuda))
    ry, rg = O.forward_grad(x, layers)
    assert y.shape == (n, 1) and gx.shape == (n, d)
    assert np.max(np.abs(y.cpu().numpy() - ry)) <= 1e-4
    assert np.max(np.abs(gx.cpu().numpy() - rg)) <= tol_rel(rg)


def test_split_zero_coords_and_no_y(cuda):
    eng = engine()
    wsx = eng.pack_split(to_dev(O.flatten(random_layers(2)), cuda))
    y, gx = eng.forward_grad_split(wsx, torch.empty(0, 2, device=cuda))
    assert y.shape == (0, 1) and gx.shape == (0, 2)
    x = torch.rand(300, 2, device=cuda) * 2 - 1
    y1, g1 = eng.forward_grad_split(wsx, x)
    y2, g2 = eng.forward_grad_split(wsx, x, want_y=False)
    assert y2 is None and torch.equal(g1, g2)


def test_split_full_size_vs_fp32_kernel_and_oracle(cuda):
    """N = 2^20 (the bench workload): a 4096-coordinate subset against the fp64 oracle, the whole batch against the
    fp32 kernel (both fp32-level, so their difference is at the fp32 rounding level), determinism."""
    layers = random_layers(2, seed=7)
    eng = engine()
    fdev = to_dev(O.flatten(layers), cuda)
    ws, wsx = eng.pack(fdev), eng.pack_split(fdev)
    g = torch.Generator(device=cuda).manual_seed(1000)
    x = torch.rand(1 << 20, 2, device=cuda, generator=g) * 2 - 1
    y, gx = eng.forward_grad_split(wsx, x)
    y2, gx2 = eng.forward_grad_split(wsx, x)
    assert torch.equal(y, y2) and torch.equal(gx, gx2)
    y32, gx32 = eng.forward_grad(ws, x)
    sc = max(1., float(gx32.abs().max()))
    assert float((y - y32).abs().max()) <= 1e-5
    assert float((gx - gx32).abs().max()) <= 1e-5 * sc
    idx = torch.arange(0, 1 << 20, 256, device=cuda)
    ry, rg = O.forward_grad(x[idx].cpu().numpy(), layers)
    assert np.max(np.abs(y[idx].cpu().numpy() - ry)) <= 1e-4
    assert np.max(np.abs(gx[idx].cpu().numpy() - rg)) <= tol_rel(rg)


def test_split_pack_tracks_weight_updates(cuda):
    """The split image is a function of the current weights (repacked per optimizer step)."""
    la, lb = random_layers(2, seed=1), random_layers(2, seed=2)
    eng = engine()
    x = torch.rand(2048, 2, device=cuda) * 2 - 1
    wa = eng.pack_split(to_dev(O.flatten(la), cuda))
    wb = eng.pack_split(to_dev(O.flatten(lb), cuda))
    _, ga = eng.forward_grad_split(wa, x)
    _, gb = eng.forward_grad_split(wb, x)
    _, rb = O.forward_grad(x.cpu().numpy(), lb)
    assert not torch.equal(ga, gb)
    assert np.max(np.abs(gb.cpu().numpy() - rb)) <= tol_rel(rb)


def test_module_precision_bf16x6(cuda, g1):
    """SingleBVPNet(precision='bf16x6') through the drop-in API: diff_operators.gradient on the jet node served by
    the split kernel matches the fp64 golden like the fp32 module, and a backward through it (fp32 recompute) agrees
    with the fp32 module's."""
    from siren_amd import diff_operators, modules
    sd = {k[2:]: np.asarray(g1[k]) for k in g1.keys() if k.startswith('w_net.')}
    ref = g1['G1_gradient_f64'][0]
    outs = {}
    for prec in ('fp32', 'bf16x6'):
        m = modules.SingleBVPNet(in_features=2, verbose=False, jet=True, precision=prec).to(cuda)
        m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
        x = to_dev(g1['coords'], cuda)
        out = m({'coords': x})
        gr = diff_operators.gradient(out['model_out'], out['model_in'])
        loss = (gr ** 2).sum()
        loss.backward()
        outs[prec] = (out['model_out'].detach().cpu().numpy()[0], gr.detach().cpu().numpy()[0],
                      m.net.net[1][0].weight.grad.detach().cpu().numpy())
    y_s, g_s, w_s = outs['bf16x6']
    y_f, g_f, w_f = outs['fp32']
    assert np.max(np.abs(g_s - ref)) <= tol_rel(ref)
    assert np.max(np.abs(y_s - g1['G1_model_out_f64'][0])) <= 1e-4
    assert np.max(np.abs(g_s - g_f)) <= 1e-5 * max(1., np.max(np.abs(g_f)))
    assert np.max(np.abs(w_s - w_f)) <= 1e-4 * np.max(np.abs(w_f))
    with pytest.raises(ValueError):
        modules.SingleBVPNet(in_features=2, verbose=False, precision='bf16')


@pytest.mark.parametrize('d', [2, 3])
@pytest.mark.parametrize('n', [1, 127, 128, 129, 4097, 70000])
def test_split_forward_ragged(cuda, n, d):
    """The forward-only split kernel (siren_forward_split, 8 waves x 16 coordinates per tile) against the fp64
    oracle's model_out."""
    layers = random_layers(d, seed=3 * n + d)
    eng = engine(d)
    wsx = eng.pack_split(to_dev(O.flatten(layers), cuda))
    x = np.random.default_rng(n + 11).uniform(-1, 1, (n, d)).astype(np.float32)
    y = eng.forward_split(wsx, to_dev(x, cuda))
    ry, _ = O.forward_grad(x, layers)
    assert y.shape == (n, 1)
    assert np.max(np.abs(y.cpu().numpy() - ry)) <= 1e-4


@pytest.mark.parametrize('name', ['g1', 'g2'])
def test_split_forward_golden_and_full_size(cuda, name, request):
    fx = request.getfixturevalue(name)
    g1 = request.getfixturevalue('g1')
    flat, _ = weights_of(fx)
    eng = engine()
    fdev = to_dev(flat, cuda)
    ws, wsx = eng.pack(fdev), eng.pack_split(fdev)
    y = eng.forward_split(wsx, to_dev(g1['coords'][0], cuda)).cpu().numpy()
    ry = fx[name.upper() + '_model_out_f64'][0]
    ey, ey32 = np.max(np.abs(y - ry)), np.max(np.abs(eng.forward(ws, to_dev(g1['coords'][0], cuda)).cpu().numpy() - ry))
    assert ey <= 1e-4 and ey <= 2 * ey32 + 1e-7
    x = torch.rand(1 << 20, 2, device=cuda) * 2 - 1
    ys, ys2, y32 = eng.forward_split(wsx, x), eng.forward_split(wsx, x), eng.forward(ws, x)
    assert torch.equal(ys, ys2)
    assert float((ys - y32).abs().max()) <= 1e-5


def test_module_precision_bf16x6_no_grad_forward_and_mesh(cuda, g1):
    """precision='bf16x6' under no_grad: model_out from the split forward kernel (vs the fp64 golden and the fp32
    module), and sdf_meshing.create_mesh's dense evaluation through it matches the fp32 module's volume."""
    from siren_amd import modules, sdf_meshing
    sd = {k[2:]: np.asarray(g1[k]) for k in g1.keys() if k.startswith('w_net.')}
    x = to_dev(g1['coords'], cuda)
    outs = {}
    for prec in ('fp32', 'bf16x6'):
        m = modules.SingleBVPNet(in_features=2, verbose=False, precision=prec).to(cuda)
        m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
        with torch.no_grad():
            outs[prec] = m({'coords': x})['model_out'].cpu().numpy()[0]
    ref = g1['G1_model_out_f64'][0]
    assert np.max(np.abs(outs['bf16x6'] - ref)) <= 1e-4
    assert np.max(np.abs(outs['bf16x6'] - outs['fp32'])) <= 1e-5
    vols = {}
    for prec in ('fp32', 'bf16x6'):
        torch.manual_seed(0)
        m = modules.SingleBVPNet(in_features=3, verbose=False, precision=prec).to(cuda)
        vols[prec] = sdf_meshing.evaluate_sdf_grid(lambda p, m=m: m({'coords': p})['model_out'], 64,
                                                    max_batch=1 << 16, device=cuda, out_device=cuda)
    assert float((vols['fp32'] - vols['bf16x6']).abs().max()) <= 1e-5


@pytest.mark.parametrize('w0,w', [(30., 10.), (3000., 30.), (10., 30.)])
@pytest.mark.parametrize('d', [2, 3])
@pytest.mark.parametrize('n', [63, 1000, 4097])
def test_split_distinct_omegas(cuda, w0, w, d, n):
    """omega_first != omega_hidden on the split kernels (separate pack-scale corrections for the first layer and the
    hidden layers): forward_grad_split and forward_split vs the fp64 oracle; the init divides by omega as the notebook
    Siren does (ipynb:71-108), so the pre-activations keep the reference's scale."""
    from siren_amd.engine import SirenEngine
    rng = np.random.default_rng(n + d + int(w0))
    dims = [d] + [256] * 4 + [1]
    layers = []
    for i, (fi, fo) in enumerate(zip(dims[:-1], dims[1:])):
        bound = 1. / fi if i == 0 else np.sqrt(6. / fi) / w
        layers.append((rng.uniform(-bound, bound, (fo, fi)).astype(np.float32),
                       (rng.uniform(-1, 1, fo) / np.sqrt(fi)).astype(np.float32)))
    eng = SirenEngine(d, 256, 3, 1, w0, w, True)
    flat = to_dev(O.flatten(layers), cuda)
    wsx = eng.pack_split(flat)
    x = np.random.default_rng(n).uniform(-1, 1, (n, d)).astype(np.float32)
    xd = to_dev(x, cuda)
    y, gx = eng.forward_grad_split(wsx, xd)
    yf = eng.forward_split(wsx, xd)
    y32, gx32 = eng.forward_grad(eng.pack(flat), xd)
    ry, rg = O.forward_grad(x, layers, omega_first=w0, omega_hidden=w)
    # the fp32 kernel's own error bounds the split's (fp32-equivalent precision mode), as at omega 30 / 30
    ey, eg = np.max(np.abs(y.cpu().numpy() - ry)), np.max(np.abs(gx.cpu().numpy() - rg))
    ey32, eg32 = np.max(np.abs(y32.cpu().numpy() - ry)), np.max(np.abs(gx32.cpu().numpy() - rg))
    assert ey <= max(1e-4, 2 * ey32) and eg <= max(tol_rel(rg), 2 * eg32 + 1e-6), (ey, eg, ey32, eg32)
    assert np.max(np.abs(yf.cpu().numpy() - ry)) <= max(1e-4, 2 * ey32)


# ---- the bf16x6 training leg: siren_backward_split (split-bf16 recompute + reverse from gy, fp32 MFMA wgrad) ----
W2_KEYS = ['net.net.%d.0.%s' % (i, k) for i in range(5) for k in ('weight', 'bias')]


def test_backward_split_vs_reference_golden(cuda, g1):
    """image_mse θ-gradients of the reference (G1, fp64) from the bf16x6 W2 backward: within the fp32 pipeline's
    tolerance and at its level of error (an fp32-equivalent mode)."""
    flat, layers = weights_of(g1)
    eng = engine()
    fdev = to_dev(flat, cuda)
    ws, wsx = eng.pack(fdev), eng.pack_split(fdev)
    x = to_dev(g1['coords'][0], cuda)
    y = eng.forward_split(wsx, x)
    gy = 2. * (y - to_dev(g1['gt_img'][0], cuda)) / y.numel()
    gx, gp = eng.backward_split(wsx, x, gy, want_gx=True)
    gx32, gp32 = eng.backward_params(ws, x, gy)
    ref = np.concatenate([g1['G1_image_mse_grad_' + k].reshape(-1) for k in W2_KEYS])
    e, e32 = np.max(np.abs(gp.cpu().numpy() - ref)), np.max(np.abs(gp32.cpu().numpy() - ref))
    print('theta-grads |d| split %.2e fp32 kernels %.2e (max |g| %.2e)' % (e, e32, np.max(np.abs(ref))))
    assert e <= 1e-4 * np.max(np.abs(ref))
    assert e <= 2 * e32 + 1e-6 * np.max(np.abs(ref))
    _, rgx = O.forward_grad(g1['coords'][0], layers, gy.cpu().numpy())
    assert np.max(np.abs(gx.cpu().numpy() - rgx)) <= 1e-4 * np.max(np.abs(rgx))
    _, gp_nogx = eng.backward_split(wsx, x, gy)  # gx not requested: the same θ-gradients
    assert torch.equal(gp_nogx, gp)


@pytest.mark.parametrize('n,d', [(1, 2), (100, 3), (5000, 2), (70000, 3)])
def test_backward_split_shapes(cuda, n, d):
    """Ragged sizes (partial tiles, one coordinate, a persistent grid's several tiles per workgroup) against fp64
    autograd of the oracle's network, and against the fp32 W2 pipeline."""
    layers = random_layers(d, seed=n)
    eng = engine(d)
    fdev = to_dev(O.flatten(layers), cuda)
    ws, wsx = eng.pack(fdev), eng.pack_split(fdev)
    rng = np.random.default_rng(n)
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    gy = (rng.normal(size=(n, 1)) / n).astype(np.float32)
    gx, gp = eng.backward_split(wsx, to_dev(x, cuda), to_dev(gy, cuda), want_gx=True)
    gx32, gp32 = eng.backward_params(ws, to_dev(x, cuda), to_dev(gy, cuda))
    xt = torch.tensor(x, dtype=torch.float64, requires_grad=True)
    params = [torch.tensor(np.asarray(t), dtype=torch.float64, requires_grad=True) for W, b in layers for t in (W, b)]
    yt = O.torch_forward(xt, params)
    g = torch.autograd.grad(yt, [xt] + params, torch.tensor(gy, dtype=torch.float64))
    rgp = torch.cat([t.reshape(-1) for t in g[1:]]).numpy()
    assert np.max(np.abs(gp.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))
    assert np.max(np.abs(gx.cpu().numpy() - g[0].numpy())) <= tol_rel(g[0].numpy())
    assert np.max(np.abs(gp.cpu().numpy() - gp32.cpu().numpy())) <= 2e-5 * np.max(np.abs(rgp))


def test_backward_split_zero_coords(cuda):
    eng = engine()
    fdev = to_dev(O.flatten(random_layers(2)), cuda)
    wsx = eng.pack_split(fdev)
    gx, gp = eng.backward_split(wsx, torch.empty(0, 2, device=cuda), torch.empty(0, 1, device=cuda), want_gx=True)
    assert gx.shape == (0, 2) and torch.count_nonzero(gp) == 0


def test_module_precision_bf16x6_training_step(cuda, g1, monkeypatch):
    """SingleBVPNet(precision='bf16x6') under image_mse training: the θ-gradients come from the stored bf16x6 split (the
    fp32 W2 entry points and the recompute form are forbidden here) and match G1's fp64 golden; y is the split forward's."""
    from siren_amd import loss_functions as Lf, modules
    from siren_amd.engine import SirenEngine

    def boom(*a, **k):
        raise AssertionError('the fp32 W2 path ran')
    for nm in ('backward_params', 'backward_stored', 'forward_store', 'forward', 'backward_split'):
        monkeypatch.setattr(SirenEngine, nm, boom)
    sd = {k[2:]: np.asarray(g1[k]) for k in g1.keys() if k.startswith('w_net.')}
    m = modules.SingleBVPNet(in_features=2, verbose=False, precision='bf16x6').to(cuda)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    out = m({'coords': to_dev(g1['coords'], cuda)})
    assert np.max(np.abs(out['model_out'].detach().cpu().numpy()[0] - g1['G1_model_out_f64'][0])) <= 1e-4
    loss = Lf.image_mse(None, out, {'img': to_dev(g1['gt_img'], cuda)})['img_loss']
    m.zero_grad()
    loss.backward()
    for k, p in m.named_parameters():
        ref = g1['G1_image_mse_grad_' + k]
        assert np.max(np.abs(p.grad.cpu().numpy() - ref)) <= 1e-4 * max(np.max(np.abs(ref)), 1e-30) + 1e-12, k


@pytest.mark.parametrize('which', ['gradients_mse', 'laplace_mse'])
def test_module_precision_bf16x6_derivative_losses(cuda, g1, monkeypatch, which):
    """SingleBVPNet(precision='bf16x6') trained through a derivative loss: the first step reaches the
    split node (SirenSplitFunction's x-derivative: SirenVJP, or fused_laplace on its node, which packs the fp32 image
    on first use), later steps the jet / Laplacian modes on the fp32 kernels. Three steps, every device-torch recompute
    forbidden: the θ-gradients match G1's fp64 golden at each step (no optimizer step in between)."""
    from siren_amd import loss_functions as Lf, modules
    forbid_torch_path(monkeypatch)
    sd = {k[2:]: np.asarray(g1[k]) for k in g1.keys() if k.startswith('w_net.')}
    m = modules.SingleBVPNet(in_features=2, verbose=False, precision='bf16x6').to(cuda)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    coords = to_dev(g1['coords'], cuda)
    for step in range(3):
        m.zero_grad()
        out = m({'coords': coords})
        if which == 'gradients_mse':
            loss = Lf.gradients_mse(out, {'gradients': to_dev(g1['gt_gradients'], cuda)})['gradients_loss']
        else:
            loss = Lf.laplace_mse(out, {'laplace': to_dev(g1['gt_laplace'], cuda)})['laplace_loss']
        loss.backward()
        for k, p in m.named_parameters():
            ref = g1['G1_%s_grad_%s' % (which, k)]
            err = np.max(np.abs(p.grad.cpu().numpy() - ref))
            assert err <= 1e-4 * max(np.max(np.abs(ref)), 1e-30) + 1e-12, (step, k, err)


def test_module_precision_bf16x6_retain_graph(cuda, g1):
    """A second backward over the same bf16x6 training graph (retain_graph=True) reads the stored split workspace
    again: the θ-gradients of the two passes are bitwise identical."""
    from siren_amd import loss_functions as Lf, modules
    sd = {k[2:]: np.asarray(g1[k]) for k in g1.keys() if k.startswith('w_net.')}
    m = modules.SingleBVPNet(in_features=2, verbose=False, precision='bf16x6').to(cuda)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    out = m({'coords': to_dev(g1['coords'], cuda)})
    loss = Lf.image_mse(None, out, {'img': to_dev(g1['gt_img'], cuda)})['img_loss']
    m.zero_grad()
    loss.backward(retain_graph=True)
    first = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
    m.zero_grad()
    loss.backward()
    for k, p in m.named_parameters():
        assert torch.equal(p.grad, first[k]), k


@pytest.mark.parametrize('n,d', [(1, 2), (100, 3), (5000, 2), (70000, 3), (1 << 18, 2)])
def test_stored_split_matches_recompute(cuda, n, d):
    """The stored bf16x6 split (forward keeps a_l / cos, reverse-only backward) against the recompute form
    (siren_backward_split) and fp64 autograd: same kernels' arithmetic, so the θ-gradients agree to the last bits
    (bitwise where the tile sums meet in the same order), and y matches the split W0."""
    layers = random_layers(d, seed=3 * n + d)
    eng = engine(d)
    fdev = to_dev(O.flatten(layers), cuda)
    wsx = eng.pack_split(fdev)
    rng = np.random.default_rng(n)
    x = to_dev(rng.uniform(-1, 1, (n, d)), cuda)
    gy = to_dev(rng.normal(size=(n, 1)) / n, cuda)
    y, tws = eng.forward_store_split(wsx, x)
    assert torch.equal(y, eng.forward_split(wsx, x))
    gx, gp = eng.backward_stored_split(wsx, x, gy, tws, want_gx=True)
    gx_r, gp_r = eng.backward_split(wsx, x, gy, want_gx=True)
    scale = float(gp_r.abs().max())
    assert float((gp - gp_r).abs().max()) <= 1e-6 * scale, float((gp - gp_r).abs().max()) / scale
    assert float((gx - gx_r).abs().max()) <= 1e-6 * max(1., float(gx_r.abs().max()))
    if n <= 5000:
        xt = torch.tensor(x.cpu().numpy(), dtype=torch.float64)
        params = [torch.tensor(np.asarray(t), dtype=torch.float64, requires_grad=True) for W, b in layers for t in (W, b)]
        yt = O.torch_forward(xt, params)
        g = torch.autograd.grad(yt, params, torch.tensor(gy.cpu().numpy(), dtype=torch.float64))
        rgp = torch.cat([t.reshape(-1) for t in g]).numpy()
        assert np.max(np.abs(gp.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))


def test_stored_split_zero_coords(cuda):
    eng = engine()
    wsx = eng.pack_split(to_dev(O.flatten(random_layers(2)), cuda))
    y, tws = eng.forward_store_split(wsx, torch.empty(0, 2, device=cuda))
    gx, gp = eng.backward_stored_split(wsx, torch.empty(0, 2, device=cuda), torch.empty(0, 1, device=cuda), tws,
                                       want_gx=True)
    assert y.shape == (0, 1) and gx.shape == (0, 2) and torch.count_nonzero(gp) == 0


def test_g5_psnr_trajectory_bf16x6(cuda, manifest, monkeypatch):
    """Config 1 in the bf16x6 training mode: 300 Adam steps on the 256^2 synthetic image through the stored split-bf16
    forward / reverse and the bf16x6 wgrad (the fp32 W2 entry points forbidden) track the reference's loss trajectory
    within 2 % and reach its PSNR within 0.05 dB, as the fp32 engine does (test_gpu_parity.py)."""
    import os
    from siren_amd.modules import SingleBVPNet
    from siren_amd import dataio
    from siren_amd.engine import SirenEngine

    def boom(*a, **k):
        raise AssertionError('the fp32 W2 path ran')
    for nm in ('backward_params', 'backward_stored', 'forward_store'):
        monkeypatch.setattr(SirenEngine, nm, boom)
    fit = dict(np.load(os.path.join(os.path.dirname(__file__), 'golden', 'golden_fit.npz')))
    torch.manual_seed(0)
    m = SingleBVPNet(verbose=False, precision='bf16x6').to(cuda)
    for k, v in m.state_dict().items():
        assert np.array_equal(v.cpu().numpy(), fit['init_' + k])
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    grid = dataio.get_mgrid(256)[None].to(cuda)
    img = dataio.synthetic_image(grid)
    losses = []
    for _ in range(300):
        out = m({'coords': grid})
        loss = ((out['model_out'] - img) ** 2).mean()
        losses.append(float(loss.detach()))
        opt.zero_grad()
        loss.backward()
        opt.step()
    with torch.no_grad():
        p = dataio.psnr(m({'coords': grid})['model_out'], img)
    ref = fit['losses']
    assert abs(p - manifest['G5_psnr_final']) < 0.05, (p, manifest['G5_psnr_final'])
    for i in range(0, 300, 10):
        assert abs(losses[i] - ref[i]) <= 0.02 * ref[i] + 1e-6, (i, losses[i], ref[i])
