"""Hidden 256 at 4..5 hidden layers (FCBlock builds any depth, /root/reference/modules.py:65-80): the derivative paths
run the stored split through HBM (siren_capi.hip deep(): MODE_FWDS + MODE_REV of the W1 kernel, tu_w1deep.hip) and
the serial W3 kernel. Parity against the reference's G12 fp64 golden (tests/golden/make_golden.py make_g12) through
the drop-in API with every device-torch recompute forbidden, and against fp64 autograd for ragged n at the engine
level. Tolerances as tests/test_gpu_parity.py. Needs an MI355X."""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as O
from conftest import forbid_torch_path, load_golden
from test_gpu_parity import random_layers, to_dev, tol_rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def g12():
    return load_golden('g12')


def _model(g12, cuda, depth, prefix=None, in_features=2, **kw):
    from siren_amd.modules import SingleBVPNet
    m = SingleBVPNet(verbose=False, in_features=in_features, num_hidden_layers=depth, **kw).to(cuda)
    p = (prefix or 'L%d' % depth) + '_w_'
    m.load_state_dict({k[len(p):]: torch.tensor(v) for k, v in g12.items() if k.startswith(p)})
    return m


@pytest.mark.parametrize('depth', [4, 5])
@pytest.mark.parametrize('jet', [False, True])
def test_forward_gradient_laplace_vs_reference(cuda, g12, depth, jet, monkeypatch):
    from siren_amd import diff_operators as D
    forbid_torch_path(monkeypatch)
    m = _model(g12, cuda, depth, jet=jet)
    eng = m.net._engine()
    assert eng.deep and eng.grad_supported and eng.second_order_supported and eng.stored_supported
    tag = 'L%d' % depth
    out = m({'coords': to_dev(g12['coords'], cuda)})
    y = out['model_out']
    assert np.max(np.abs(y.detach().cpu().numpy() - g12[tag + '_model_out_f64'])) <= 1e-4
    g = D.gradient(y, out['model_in'])
    assert np.max(np.abs(g.detach().cpu().numpy() - g12[tag + '_gradient_f64'])) <= tol_rel(g12[tag + '_gradient_f64'])
    lap = D.laplace(y, out['model_in'])
    assert np.max(np.abs(lap.detach().cpu().numpy() - g12[tag + '_laplace_f64'])) <= tol_rel(g12[tag + '_laplace_f64'])


@pytest.mark.parametrize('depth', [4, 5])
@pytest.mark.parametrize('loss', ['image_mse', 'gradients_mse', 'laplace_mse'])
def test_training_theta_grads_vs_reference(cuda, g12, depth, loss, monkeypatch):
    """The three image-family losses (loss_functions.py:8-12, 84-109) train a 4- / 5-hidden-layer net on kernels."""
    from siren_amd import loss_functions as Lf
    forbid_torch_path(monkeypatch)
    m = _model(g12, cuda, depth)
    tag = 'L%d' % depth
    gt = {'img': to_dev(g12['gt_img'], cuda), 'gradients': to_dev(g12['gt_gradients'], cuda),
          'laplace': to_dev(g12['gt_laplace'], cuda)}
    for _ in range(2):  # the second pass runs with jet mode switched on (SirenJetFunction / kept forward)
        out = m({'coords': to_dev(g12['coords'], cuda)})
        fn = getattr(Lf, loss)
        losses = fn(None, out, gt) if loss == 'image_mse' else fn(out, gt)
        total = sum(v.mean() for v in losses.values())
        m.zero_grad()
        total.backward()
        for k, p in m.named_parameters():
            ref = g12['%s_%s_grad_%s' % (tag, loss, k)]
            got = p.grad.cpu().numpy() if p.grad is not None else np.zeros_like(ref)
            assert np.max(np.abs(got - ref)) <= 1e-4 * max(np.max(np.abs(ref)), 1e-30) + 1e-12, (k, loss)


def test_sdf_depth5_vs_reference(cuda, g12, manifest, monkeypatch):
    """sdf (loss_functions.py:214-238) on a 5-hidden-layer d3 net: value + gradient terms, the kept W3 on the deep
    stored forward, fp64 theta-grads of the reference."""
    from siren_amd import loss_functions as Lf
    forbid_torch_path(monkeypatch)
    m = _model(g12, cuda, 5, prefix='S5', in_features=3)
    for _ in range(2):
        out = m({'coords': to_dev(g12['S5_coords'], cuda)})
        terms = Lf.sdf(out, {'sdf': to_dev(g12['S5_gt_sdf'], cuda), 'normals': to_dev(g12['S5_gt_normals'], cuda)})
        for k, v in terms.items():
            ref = manifest['G12_S5_sdf_%s_f64' % k]
            assert abs(float(v.detach()) - ref) <= 1e-4 * max(1., abs(ref)), k
        total = sum(v.mean() for v in terms.values())
        m.zero_grad()
        total.backward()
        for k, p in m.named_parameters():
            ref = g12['S5_sdf_grad_' + k]
            assert np.max(np.abs(p.grad.cpu().numpy() - ref)) <= 1e-4 * np.max(np.abs(ref)) + 1e-12, k


@pytest.mark.parametrize('n,d,L,o', [(1, 2, 4, 1), (65, 3, 5, 2), (4097, 2, 5, 1), (333, 1, 4, 3), (0, 2, 4, 1)])
def test_engine_w1_w2_vs_fp64(cuda, n, d, L, o):
    """siren_forward_grad (W1) and siren_backward (W2) at 4..5 hidden layers against the fp64 oracle / autograd,
    ragged n; the stored split (forward_store + backward_stored) equals siren_backward bitwise."""
    from siren_amd.engine import SirenEngine
    layers = random_layers(d, L, o, seed=n + 7 * L)
    eng = SirenEngine(d, 256, L, o)
    assert eng.deep and eng.grad_supported and eng.stored_supported
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n + d)
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    gy = rng.normal(size=(n, o)).astype(np.float32)
    xd, gyd = to_dev(x, cuda).reshape(n, d), to_dev(gy, cuda).reshape(n, o)
    y, gx = eng.forward_grad(ws, xd, gyd)
    gxb, gp = eng.backward_params(ws, xd, gyd)
    torch.cuda.synchronize()
    if n == 0:
        assert gp.abs().max() == 0
        return
    xt = torch.tensor(x, dtype=torch.float64, requires_grad=True)
    params = [torch.tensor(t, dtype=torch.float64, requires_grad=True) for W, b in layers for t in (W, b)]
    yt = O.torch_forward(xt, params)
    grads = torch.autograd.grad(yt, [xt] + params, torch.tensor(gy, dtype=torch.float64))
    rgx = grads[0].numpy()
    rgp = torch.cat([g.reshape(-1) for g in grads[1:]]).numpy()
    assert np.max(np.abs(y.cpu().numpy() - yt.detach().numpy())) <= 1e-4
    assert np.max(np.abs(gx.cpu().numpy() - rgx)) <= tol_rel(rgx)
    assert torch.equal(gx, gxb)
    assert np.max(np.abs(gp.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))
    y2, tws = eng.forward_store(ws, xd)
    gx2, gp2 = eng.backward_stored(ws, xd, gyd, tws)
    assert torch.equal(y2, y) and torch.equal(gx2, gxb) and torch.equal(gp2, gp)


@pytest.mark.parametrize('n,d,L,o,theta', [(300, 2, 4, 1, True), (1000, 3, 5, 1, True), (77, 2, 5, 3, False)])
def test_engine_second_order_vs_fp64(cuda, n, d, L, o, theta):
    """W3 (the serial kernel's layer loops) at 4..5 hidden layers: H v and the mixed theta-gradient vs fp64."""
    from siren_amd.engine import SirenEngine
    layers = random_layers(d, L, o, seed=3 * n + L)
    eng = SirenEngine(d, 256, L, o)
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n)
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    v = rng.normal(size=(n, d)).astype(np.float32)
    gx, gp = eng.second_order(ws, to_dev(x, cuda), to_dev(v, cuda), want_theta=theta)
    xt = torch.tensor(x, dtype=torch.float64, requires_grad=True)
    params = [torch.tensor(t, dtype=torch.float64, requires_grad=True) for W, b in layers for t in (W, b)]
    yt = O.torch_forward(xt, params)
    J = torch.autograd.grad(yt, xt, torch.ones_like(yt), create_graph=True)[0]
    S = (J * torch.tensor(v, dtype=torch.float64)).sum()
    grads = torch.autograd.grad(S, [xt] + params, allow_unused=True)  # b_out does not reach J
    grads = [torch.zeros_like(p) if g is None else g for g, p in zip(grads, [xt] + params)]
    rgx = grads[0].numpy()
    assert np.max(np.abs(gx.cpu().numpy() - rgx)) <= 1e-4 * max(1., np.max(np.abs(rgx)))
    if theta:
        rgp = torch.cat([g.reshape(-1) for g in grads[1:]]).numpy()
        assert np.max(np.abs(gp.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))
