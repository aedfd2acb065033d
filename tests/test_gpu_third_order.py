"""Third-order adjoint on the HIP kernels: the backward of the Hessian-vector-product node (siren_hvp_backward, the
mixed jet of jet_kernel.hpp) against fp64 autograd, and the reference's own laplace_mse recipe —
laplace = divergence(gradient(y, x)) with one create_graph autograd.grad per input dimension
(/root/reference/diff_operators.py:27-43, loss_functions.py:104-109) — trained end to end with every device-torch
recompute of siren_amd._torch_path forbidden, against the reference's G1 / G2 laplace_mse theta-gradients.
Needs an MI355X.

Tolerances: derivatives abs <= 1e-4 * max(1, max|ref|) (gx, gv, gu), theta-grads abs <= 1e-4 *
max|ref|, all against fp64 references.
"""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as O
from conftest import forbid_torch_path

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


def hvp_vjp_ref(x, layers, v, g, u):
    """fp64 autograd of S = sum <g, sum_j u_j H_j v>: returns dS/dx, dS/dtheta, dS/dv, dS/du."""
    xt = torch.tensor(x, dtype=torch.float64, requires_grad=True)
    params = [torch.tensor(t, dtype=torch.float64, requires_grad=True) for W, b in layers for t in (W, b)]
    vt = torch.tensor(v, dtype=torch.float64, requires_grad=True)
    y = O.torch_forward(xt, params)
    ut = (torch.ones_like(y) if u is None else torch.tensor(u, dtype=torch.float64)).requires_grad_(True)
    Ju = torch.autograd.grad(y, xt, ut, create_graph=True)[0]
    hv = torch.autograd.grad(Ju, xt, vt, create_graph=True)[0]
    S = (hv * torch.tensor(g, dtype=torch.float64)).sum()
    grads = torch.autograd.grad(S, [xt, vt, ut] + params, allow_unused=True)
    gp = torch.cat([(torch.zeros_like(p) if gg is None else gg).reshape(-1) for gg, p in zip(grads[3:], params)])
    return grads[0].numpy(), gp.numpy(), grads[1].numpy(), grads[2].numpy()


@pytest.mark.parametrize('n,d,L,o,weighted', [(1, 2, 3, 1, False), (15, 2, 3, 1, False), (4097, 2, 3, 1, False),
                                               (1000, 3, 3, 1, True), (333, 3, 2, 3, True), (700, 4, 1, 2, True),
                                               (2048, 2, 3, 2, True), (300, 1, 5, 1, False), (65, 2, 4, 4, True)])
def test_hvp_backward_vs_fp64(cuda, n, d, L, o, weighted):
    from siren_amd.engine import SirenEngine
    layers = random_layers(d, L, o, seed=7 * n + L + o)
    eng = SirenEngine(d, 256, L, o)
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n + d)
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    v = rng.normal(size=(n, d)).astype(np.float32)
    g = (rng.normal(size=(n, d)) / n).astype(np.float32)
    u = rng.normal(size=(n, o)).astype(np.float32) if weighted else None
    gx, gp, gv, gu = eng.hvp_backward(ws, to_dev(x, cuda), to_dev(v, cuda), to_dev(g, cuda),
                                      to_dev(u, cuda) if weighted else None, want_theta=True, want_v=True,
                                      want_u=True)
    rgx, rgp, rgv, rgu = hvp_vjp_ref(x, layers, v, g, u)
    assert np.max(np.abs(gp.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))
    assert np.max(np.abs(gx.cpu().numpy() - rgx)) <= 1e-4 * max(1e-6, np.max(np.abs(rgx)))
    assert np.max(np.abs(gv.cpu().numpy() - rgv)) <= 1e-4 * max(1e-6, np.max(np.abs(rgv)))
    assert np.max(np.abs(gu.cpu().numpy() - rgu)) <= 1e-4 * max(1e-6, np.max(np.abs(rgu)))
    # the optional outputs do not change the others (x only request: no theta / v / u work)
    gx2, none_p, none_v, none_u = eng.hvp_backward(ws, to_dev(x, cuda), to_dev(v, cuda), to_dev(g, cuda),
                                                   to_dev(u, cuda) if weighted else None, want_theta=False)
    assert none_p is None and none_v is None and none_u is None and torch.equal(gx, gx2)


def test_hvp_backward_n0_and_determinism(cuda):
    from siren_amd.engine import SirenEngine
    from siren_amd import dataio
    layers = random_layers(2, 3, 1, seed=3)
    eng = SirenEngine(2, 256, 3, 1)
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    z = torch.empty(0, 2, device=cuda)
    gx, gp, _, _ = eng.hvp_backward(ws, z, z, z)
    assert gx.shape == (0, 2) and float(gp.abs().max()) == 0.
    x = dataio.get_mgrid(512).to(cuda)  # config-5 size
    v = torch.zeros_like(x)
    v[:, 0] = 1.
    g = torch.randn_like(x) / x.shape[0]
    a = eng.hvp_backward(ws, x, v, g)
    b = eng.hvp_backward(ws, x, v, g)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    c = eng.hvp_backward(ws, x, v, 2. * g)  # linear in the cotangent
    assert torch.allclose(c[1], 2. * a[1], rtol=0, atol=1e-5 * float(a[1].abs().max()))
    idx = torch.randperm(x.shape[0], generator=torch.Generator().manual_seed(0))[:512]
    rgx, _, _, _ = hvp_vjp_ref(x[idx].cpu().numpy(), layers, v[idx].cpu().numpy(), g[idx].cpu().numpy(), None)
    assert np.max(np.abs(a[0][idx].cpu().numpy() - rgx)) <= 1e-4 * max(1e-6, np.max(np.abs(rgx)))


def reference_laplace(y, x):
    """The reference's op sequence (diff_operators.py:27-43): gradient with create_graph, then one create_graph
    autograd.grad per input dimension — NOT siren_amd.diff_operators.laplace's fused interception."""
    grad = torch.autograd.grad(y, [x], grad_outputs=torch.ones_like(y), create_graph=True)[0]
    div = 0.
    for i in range(grad.shape[-1]):
        div += torch.autograd.grad(grad[..., i], x, torch.ones_like(grad[..., i]), create_graph=True)[0][..., i:i + 1]
    return div


@pytest.mark.parametrize('name', ['g1', 'g2'])
def test_reference_recipe_laplace_mse_trains_on_kernels(cuda, g1, name, request, monkeypatch):
    """laplace_mse with the untouched recipe: gradient -> per-dimension divergence -> backward(), twice (the first
    pass records SirenVJP nodes, the second runs with jet mode switched on: SirenJetFunction), every _torch_path
    function forbidden; theta-grads vs the reference's fp64 laplace_mse gradients."""
    from siren_amd.modules import SingleBVPNet
    fx = request.getfixturevalue(name)
    tag = name.upper()
    forbid_torch_path(monkeypatch)
    m = SingleBVPNet(verbose=False).to(cuda)
    m.load_state_dict({k[2:]: torch.tensor(v) for k, v in fx.items() if k.startswith('w_')})
    gt = to_dev(g1['gt_laplace'], cuda)
    for _ in range(2):
        m.zero_grad()
        out = m({'coords': to_dev(g1['coords'], cuda)})
        lap = reference_laplace(out['model_out'], out['model_in'])
        loss = torch.mean((lap - gt) ** 2)  # loss_functions.py:104-109
        loss.backward()
        rl = fx[tag + '_laplace_f64']
        assert np.max(np.abs(lap.detach().cpu().numpy() - rl)) <= tol_rel(rl)
        for k, p in m.named_parameters():
            ref = fx[tag + '_laplace_mse_grad_' + k]
            assert np.max(np.abs(p.grad.cpu().numpy() - ref)) <= 1e-4 * np.max(np.abs(ref)) + 1e-12, k


def test_reference_recipe_laplace_mse_matches_fused(cuda, g2):
    """The two HIP routes to the same loss gradient agree: the reference recipe (d HVP nodes -> d mixed jets) and
    the fused W4 / W4s node."""
    from siren_amd import loss_functions as LF
    from siren_amd.modules import SingleBVPNet
    coords = (torch.rand(1, 5000, 2, generator=torch.Generator().manual_seed(4)) * 2 - 1).to(cuda)
    gt = torch.sin(3 * coords[..., :1]) * 1e3
    grads = []
    for fused in (False, True):
        m = SingleBVPNet(verbose=False).to(cuda)
        m.load_state_dict({k[2:]: torch.tensor(v) for k, v in g2.items() if k.startswith('w_')})
        out = m({'coords': coords})
        if fused:
            loss = LF.laplace_mse(out, {'laplace': gt})['laplace_loss']
        else:
            loss = torch.mean((reference_laplace(out['model_out'], out['model_in']) - gt) ** 2)
        loss.backward()
        grads.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]))
    assert float((grads[0] - grads[1]).abs().max()) <= 2e-5 * float(grads[1].abs().max())


def random_layers_h(d, L, o, H, seed=0, w=30.):
    rng = np.random.default_rng(seed)
    dims = [d] + [H] * (L + 1) + [o]
    layers = []
    for i, (fi, fo) in enumerate(zip(dims[:-1], dims[1:])):
        bound = 1. / fi if i == 0 else np.sqrt(6. / fi) / w
        layers.append((rng.uniform(-bound, bound, (fo, fi)).astype(np.float32),
                       (rng.uniform(-1, 1, fo) / np.sqrt(fi)).astype(np.float32)))
    return layers


@pytest.mark.parametrize('n,d,L,o,weighted', [(1, 2, 3, 1, False), (777, 3, 3, 3, True), (2000, 2, 1, 1, False),
                                               (65, 4, 4, 2, True)])
def test_hvp_backward_hidden512_vs_fp64(cuda, n, d, L, o, weighted):
    """The third-order adjoint at hidden 512 (wide_jet_kernel<4>: the four-stream mixed jet, 4 coordinates per
    wave) against fp64 autograd."""
    from siren_amd.engine import SirenEngine
    layers = random_layers_h(d, L, o, 512, seed=11 * n + L)
    eng = SirenEngine(d, 512, L, o)
    assert eng.hvp_backward_supported
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n + 7)
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    v = rng.normal(size=(n, d)).astype(np.float32)
    g = (rng.normal(size=(n, d)) / n).astype(np.float32)
    u = rng.normal(size=(n, o)).astype(np.float32) if weighted else None
    gx, gp, gv, gu = eng.hvp_backward(ws, to_dev(x, cuda), to_dev(v, cuda), to_dev(g, cuda),
                                      to_dev(u, cuda) if weighted else None, want_theta=True, want_v=True,
                                      want_u=True)
    rgx, rgp, rgv, rgu = hvp_vjp_ref(x, layers, v, g, u)
    assert np.max(np.abs(gp.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))
    assert np.max(np.abs(gx.cpu().numpy() - rgx)) <= 1e-4 * max(1e-6, np.max(np.abs(rgx)))
    assert np.max(np.abs(gv.cpu().numpy() - rgv)) <= 1e-4 * max(1e-6, np.max(np.abs(rgv)))
    assert np.max(np.abs(gu.cpu().numpy() - rgu)) <= 1e-4 * max(1e-6, np.max(np.abs(rgu)))


def test_reference_recipe_laplace_mse_hidden512_on_kernels(cuda, monkeypatch):
    """laplace_mse at hidden_features=512 through the reference's divergence(gradient()) with every torch recompute
    forbidden: W1 / W3 (two-stream jet) / third-order (mixed jet) kernels at hidden 512, theta-grads vs fp64
    autograd of the same loss (oracle restatement, modules.py + diff_operators.py op sequence)."""
    from siren_amd.modules import SingleBVPNet
    forbid_torch_path(monkeypatch)
    torch.manual_seed(0)
    m = SingleBVPNet(hidden_features=512, verbose=False).to(cuda)
    coords = (torch.rand(1, 700, 2, generator=torch.Generator().manual_seed(5)) * 2 - 1)
    gt = torch.sin(4 * coords[..., :1]) * 100.
    params64 = [p.detach().cpu().double().requires_grad_(True) for p in m.parameters()]
    x64 = coords[0].double().requires_grad_(True)
    lap64 = O.torch_laplace(O.torch_forward(x64, params64), x64)
    loss64 = torch.mean((lap64 - gt[0].double()) ** 2)
    ref = [torch.zeros_like(p) if r is None else r
           for r, p in zip(torch.autograd.grad(loss64, params64, allow_unused=True), params64)]  # b_out: unused
    for _ in range(2):
        m.zero_grad()
        out = m({'coords': coords.to(cuda)})
        loss = torch.mean((reference_laplace(out['model_out'], out['model_in']) - gt.to(cuda)) ** 2)
        loss.backward()
        assert abs(float(loss.detach()) - float(loss64.detach())) <= 1e-4 * max(1., float(loss64.detach()))
        for (k, p), r in zip(m.named_parameters(), ref):
            r = r.numpy()
            assert np.max(np.abs(p.grad.cpu().numpy() - r)) <= 1e-4 * np.max(np.abs(r)) + 1e-12, k


def hessian_vjp_ref(x, layers, G, u):
    """fp64 autograd of S = sum_c <G_c, Hm_c>, Hm[c, :, i] = sum_j u_j H_j(x_c) e_i: dS/dx, dS/dtheta, dS/du."""
    xt = torch.tensor(x, dtype=torch.float64, requires_grad=True)
    params = [torch.tensor(t, dtype=torch.float64, requires_grad=True) for W, b in layers for t in (W, b)]
    y = O.torch_forward(xt, params)
    ut = (torch.ones_like(y) if u is None else torch.tensor(u, dtype=torch.float64)).requires_grad_(True)
    Ju = torch.autograd.grad(y, xt, ut, create_graph=True)[0]
    Gt = torch.tensor(G, dtype=torch.float64)
    S = 0.
    for i in range(x.shape[1]):
        e = torch.zeros_like(Ju)
        e[:, i] = 1.
        S = S + (torch.autograd.grad(Ju, xt, e, create_graph=True)[0] * Gt[:, :, i]).sum()
    grads = torch.autograd.grad(S, [xt, ut] + params, allow_unused=True)
    gp = torch.cat([(torch.zeros_like(p) if gg is None else gg).reshape(-1) for gg, p in zip(grads[2:], params)])
    return grads[0].numpy(), gp.numpy(), grads[1].numpy()


@pytest.mark.parametrize('n,d,L,o,weighted', [(1, 2, 3, 1, False), (15, 2, 3, 1, False), (4097, 2, 3, 1, False),
                                               (333, 1, 2, 3, True), (700, 2, 1, 2, True), (2048, 2, 3, 2, True),
                                               (300, 1, 5, 1, False), (65, 2, 4, 4, True), (1000, 2, 5, 1, True)])
def test_hessian_backward_vs_fp64(cuda, n, d, L, o, weighted):
    """siren_hessian_backward (the quadratic-form jet: one sweep for the whole Hessian node's cotangent G, any
    non-symmetric G, optional output weighting u) against fp64 autograd; and the node's forward (the Hessian)."""
    from siren_amd.engine import SirenEngine
    layers = random_layers(d, L, o, seed=5 * n + L + o)
    eng = SirenEngine(d, 256, L, o)
    assert eng.hessian_backward_supported
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n + 3 * d)
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    G = (rng.normal(size=(n, d, d)) / n).astype(np.float32)
    u = rng.normal(size=(n, o)).astype(np.float32) if weighted else None
    ud = to_dev(u, cuda) if weighted else None
    gx, gp, gu = eng.hessian_backward(ws, to_dev(x, cuda), to_dev(G, cuda), ud, want_theta=True, want_u=True)
    rgx, rgp, rgu = hessian_vjp_ref(x, layers, G, u)
    assert np.max(np.abs(gp.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))
    assert np.max(np.abs(gx.cpu().numpy() - rgx)) <= 1e-4 * max(1e-6, np.max(np.abs(rgx)))
    assert np.max(np.abs(gu.cpu().numpy() - rgu)) <= 1e-4 * max(1e-6, np.max(np.abs(rgu)))
    gx2, none_p, none_u = eng.hessian_backward(ws, to_dev(x, cuda), to_dev(G, cuda), ud, want_theta=False)
    assert none_p is None and none_u is None and torch.equal(gx, gx2)
    # the node's forward (siren_hessian, one 6-stream jet sweep): Hm[:, :, i] = sum_j u_j H_j e_i; with its kept
    # jets the backward skips its forward GEMMs (siren_hessian_backward_kept) — same bar against fp64
    hm0 = eng.hessian(ws, to_dev(x, cuda), ud)
    hmk, kept = eng.hessian(ws, to_dev(x, cuda), ud, keep=True)
    assert torch.equal(hm0, hmk) and torch.isfinite(kept).all()
    kx, kp, ku = eng.hessian_backward(ws, to_dev(x, cuda), to_dev(G, cuda), ud, want_theta=True, want_u=True,
                                      kept=kept)
    assert np.max(np.abs(kp.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))
    assert np.max(np.abs(kx.cpu().numpy() - rgx)) <= 1e-4 * max(1e-6, np.max(np.abs(rgx)))
    assert np.max(np.abs(ku.cpu().numpy() - rgu)) <= 1e-4 * max(1e-6, np.max(np.abs(rgu)))
    hm = hm0.cpu().numpy()
    assert np.array_equal(hm, np.swapaxes(hm, 1, 2))  # symmetric by construction (H_12 written twice)
    xt = torch.tensor(x, dtype=torch.float64, requires_grad=True)
    params = [torch.tensor(t, dtype=torch.float64) for W, b in layers for t in (W, b)]
    y = O.torch_forward(xt, params)
    Ju = torch.autograd.grad(y, xt, torch.ones_like(y) if u is None else torch.tensor(u, dtype=torch.float64),
                             create_graph=True)[0]
    for i in range(d):
        e = torch.zeros_like(Ju)
        e[:, i] = 1.
        ref = torch.autograd.grad(Ju, xt, e, retain_graph=True)[0].numpy()
        assert np.max(np.abs(hm[:, :, i] - ref)) <= 1e-4 * max(1., np.max(np.abs(ref)))


@pytest.mark.parametrize('n,d,L,o,weighted', [(1, 2, 3, 1, False), (4097, 2, 3, 1, False), (333, 1, 2, 3, True),
                                               (1000, 2, 1, 2, True), (70, 2, 4, 4, True), (2500, 2, 5, 1, True),
                                               (65536, 2, 3, 1, False)])
def test_hessian_backward_interleaved_vs_serial(cuda, n, d, L, o, weighted):
    """The interleaved kept backward (qfi_rev_kernel, default) against the serial one (qf_rev_kernel,
    SIREN_FLAG_QF_SERIAL): the same per-element arithmetic (qf_elem) on a different schedule, so gx and gu agree
    bitwise and the theta-grads to rounding (non-symmetric G, 1..5 hidden layers, ragged n)."""
    from siren_amd.engine import SirenEngine
    layers = random_layers(d, L, o, seed=7 * n + L)
    eng, ser = SirenEngine(d, 256, L, o), SirenEngine(d, 256, L, o, flags=8)
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n + 1)
    x = to_dev(rng.uniform(-1, 1, (n, d)).astype(np.float32), cuda)
    G = to_dev((rng.normal(size=(n, d, d)) / max(n, 1)).astype(np.float32), cuda)
    u = to_dev(rng.normal(size=(n, o)).astype(np.float32), cuda) if weighted else None
    _, kept = eng.hessian(ws, x, u, keep=True)
    a = eng.hessian_backward(ws, x, G, u, want_theta=True, want_u=True, kept=kept)
    b = ser.hessian_backward(ws, x, G, u, want_theta=True, want_u=True, kept=kept)
    assert torch.equal(a[0], b[0]), float((a[0] - b[0]).abs().max())  # gx
    assert torch.equal(a[2], b[2]), float((a[2] - b[2]).abs().max())  # gu
    assert torch.isfinite(a[1]).all()
    assert float((a[1] - b[1]).abs().max()) <= 1e-6 * float(b[1].abs().max())
    c = eng.hessian_backward(ws, x, G, u, want_theta=True, want_u=True, kept=kept)
    assert all(torch.equal(p, q) for p, q in zip(a, c))  # deterministic


def test_hessian_node_forward_matches_w3_axes(cuda):
    """siren_hessian (forward-mode 6-stream jet) against the W3 reverse-over-forward sweep along each axis (the
    node's previous forward): two independent second-order methods agree to fp32 rounding."""
    from siren_amd.engine import SirenEngine
    for n, d, L, o, weighted in [(5000, 2, 3, 1, False), (77, 1, 2, 2, True), (1031, 2, 1, 3, True)]:
        layers = random_layers(d, L, o, seed=n)
        eng = SirenEngine(d, 256, L, o)
        ws = eng.pack(to_dev(O.flatten(layers), cuda))
        x = (torch.rand(n, d, device=cuda) * 2 - 1)
        u = torch.randn(n, o, device=cuda) if weighted else None
        hm = eng.hessian(ws, x, u)
        for i in range(d):
            v = torch.zeros(n, d, device=cuda)
            v[:, i] = 1.
            col = eng.second_order(ws, x, v, want_theta=False, u=u)[0]
            assert (hm[:, :, i] - col).abs().max() <= 2e-5 * max(1., float(col.abs().max())), (n, d, i)


def test_reference_recipe_runs_one_hessian_backward(cuda, monkeypatch):
    """The reference's divergence(gradient()) records d Hessian products of ONE shared SirenHessian node, so the
    backward runs siren_hessian_backward once per step (not d mixed-jet sweeps)."""
    from siren_amd.engine import SirenEngine
    from siren_amd.modules import SingleBVPNet
    calls = {'hess': 0, 'hvp': 0}
    orig_h, orig_v = SirenEngine.hessian_backward, SirenEngine.hvp_backward

    def hess(self, *a, **k):
        calls['hess'] += 1
        return orig_h(self, *a, **k)

    def hvp(self, *a, **k):
        calls['hvp'] += 1
        return orig_v(self, *a, **k)
    monkeypatch.setattr(SirenEngine, 'hessian_backward', hess)
    monkeypatch.setattr(SirenEngine, 'hvp_backward', hvp)
    torch.manual_seed(0)
    m = SingleBVPNet(verbose=False).to(cuda)
    coords = (torch.rand(1, 1000, 2) * 2 - 1).to(cuda)
    for step in range(2):  # SirenVJP nodes, then jet mode (SirenJetFunction)
        out = m({'coords': coords})
        loss = torch.mean(reference_laplace(out['model_out'], out['model_in']) ** 2)
        loss.backward()
        assert calls == {'hess': step + 1, 'hvp': 0}


def test_reference_recipe_one_forward_sweep(cuda, g1, monkeypatch):
    """From the third step on (a Hessian node was built from the jet node: JetState.hessian) the jet forward IS the
    Hessian node's sweep (siren_hessian_ex: y, dPhi/dx, Hm, kept): no W1 forward, no second Hessian forward, one kept
    backward — and the step still matches the reference's fp64 laplace_mse theta-grads (G1) and its Laplacian."""
    from siren_amd.engine import SirenEngine
    from siren_amd.modules import SingleBVPNet
    forbid_torch_path(monkeypatch)
    calls = {'w1': 0, 'hess': 0, 'hess_yg': 0, 'bwd_kept': 0}
    orig_fg, orig_fgs, orig_h, orig_b = (SirenEngine.forward_grad, SirenEngine.forward_grad_store,
                                         SirenEngine.hessian, SirenEngine.hessian_backward)

    def fg(self, *a, **k):
        calls['w1'] += 1
        return orig_fg(self, *a, **k)

    def fgs(self, *a, **k):
        calls['w1'] += 1
        return orig_fgs(self, *a, **k)

    def hess(self, *a, **k):
        calls['hess_yg' if k.get('want_yg') else 'hess'] += 1
        return orig_h(self, *a, **k)

    def bwd(self, *a, **k):
        calls['bwd_kept'] += k.get('kept') is not None
        return orig_b(self, *a, **k)
    monkeypatch.setattr(SirenEngine, 'forward_grad', fg)
    monkeypatch.setattr(SirenEngine, 'forward_grad_store', fgs)
    monkeypatch.setattr(SirenEngine, 'hessian', hess)
    monkeypatch.setattr(SirenEngine, 'hessian_backward', bwd)
    m = SingleBVPNet(verbose=False).to(cuda)
    m.load_state_dict({k[2:]: torch.tensor(v) for k, v in g1.items() if k.startswith('w_')})
    gt = to_dev(g1['gt_laplace'], cuda)
    for step in range(3):
        for k in calls:
            calls[k] = 0
        m.zero_grad()
        out = m({'coords': to_dev(g1['coords'], cuda)})
        lap = reference_laplace(out['model_out'], out['model_in'])
        torch.mean((lap - gt) ** 2).backward()
        if step == 2:
            assert calls == {'w1': 0, 'hess': 0, 'hess_yg': 1, 'bwd_kept': 1}, calls
            rl = g1['G1_laplace_f64']
            assert np.max(np.abs(lap.detach().cpu().numpy() - rl)) <= tol_rel(rl)
            for k, p in m.named_parameters():
                ref = g1['G1_laplace_mse_grad_' + k]
                assert np.max(np.abs(p.grad.cpu().numpy() - ref)) <= 1e-4 * np.max(np.abs(ref)) + 1e-12, k
            y = out['model_out'].detach().cpu().numpy()
            assert np.max(np.abs(y - g1['G1_model_out_f64'])) <= 1e-4
    # the loss stops asking for the Hessian (a first-order gradient loss): one wasted speculative sweep, then the
    # jet forward is the W1 kernel again
    from siren_amd import diff_operators as D
    for step in range(3):
        for k in calls:
            calls[k] = 0
        out = m({'coords': to_dev(g1['coords'], cuda)})
        g = D.gradient(out['model_out'], out['model_in'])
        m.zero_grad()
        (g ** 2).mean().backward()
        if step >= 1:
            assert calls['hess_yg'] == 0 and calls['w1'] == 1, (step, calls)


def test_speculation_is_tracked_per_call(cuda, g1, monkeypatch):
    """A module called twice per step (here a training batch whose Laplacian is taken through the reference recipe,
    and a smaller batch with a first-order loss) keeps the Hessian-node speculation for the consuming call only
    (JetState keys its cells by the call's coordinate shape): from the third step on, the training call runs one
    Hessian sweep (y, dPhi/dx, Hm at once), the other call one W1 launch, and no sweep is wasted; the training call's
    theta-grads still match the reference's fp64 laplace_mse gradients (G1)."""
    from siren_amd import diff_operators as D
    from siren_amd.engine import SirenEngine
    from siren_amd.modules import SingleBVPNet
    forbid_torch_path(monkeypatch)
    calls = {'w1': 0, 'hess_yg': 0}
    orig_fg, orig_fgs, orig_h = SirenEngine.forward_grad, SirenEngine.forward_grad_store, SirenEngine.hessian

    def fg(self, *a, **k):
        calls['w1'] += 1
        return orig_fg(self, *a, **k)

    def fgs(self, *a, **k):
        calls['w1'] += 1
        return orig_fgs(self, *a, **k)

    def hess(self, *a, **k):
        calls['hess_yg'] += bool(k.get('want_yg'))
        return orig_h(self, *a, **k)
    monkeypatch.setattr(SirenEngine, 'forward_grad', fg)
    monkeypatch.setattr(SirenEngine, 'forward_grad_store', fgs)
    monkeypatch.setattr(SirenEngine, 'hessian', hess)
    m = SingleBVPNet(verbose=False).to(cuda)
    m.load_state_dict({k[2:]: torch.tensor(v) for k, v in g1.items() if k.startswith('w_')})
    gt = to_dev(g1['gt_laplace'], cuda)
    other = (torch.rand(1, 300, 2, generator=torch.Generator().manual_seed(5)) * 2 - 1).to(cuda)
    for step in range(4):
        for k in calls:
            calls[k] = 0
        m.zero_grad()
        out = m({'coords': to_dev(g1['coords'], cuda)})
        lap = reference_laplace(out['model_out'], out['model_in'])
        loss = torch.mean((lap - gt) ** 2)
        loss.backward()
        grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
        m.zero_grad()
        o2 = m({'coords': other})
        (D.gradient(o2['model_out'], o2['model_in']) ** 2).mean().backward()
        if step >= 2:
            assert calls == {'w1': 1, 'hess_yg': 1}, (step, calls)
            for k, gk in grads.items():
                ref = g1['G1_laplace_mse_grad_' + k]
                assert np.max(np.abs(gk.cpu().numpy() - ref)) <= 1e-4 * np.max(np.abs(ref)) + 1e-12, k


@pytest.mark.parametrize('n,d,L,o,weighted', [(1, 2, 3, 1, False), (1000, 2, 3, 1, False), (333, 1, 2, 3, True),
                                               (4097, 2, 5, 2, True), (70, 2, 4, 4, True)])
def test_hessian_ex_value_and_gradient(cuda, n, d, L, o, weighted):
    """siren_hessian_ex: y and the seed-weighted gradient from the Hessian sweep against the W1 kernel
    (siren_forward_grad with gy = u) and fp64 autograd; Hm and the kept jets bitwise those of siren_hessian."""
    from siren_amd.engine import SirenEngine
    layers = random_layers(d, L, o, seed=n + 13 * L)
    eng = SirenEngine(d, 256, L, o)
    ws = eng.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(n)
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    u = rng.normal(size=(n, o)).astype(np.float32) if weighted else None
    xd, ud = to_dev(x, cuda), (to_dev(u, cuda) if weighted else None)
    hm, kept, y, g = eng.hessian(ws, xd, ud, keep=True, want_yg=True)
    hm0, kept0 = eng.hessian(ws, xd, ud, keep=True)
    assert torch.equal(hm, hm0) and torch.equal(kept, kept0)
    xt = torch.tensor(x, dtype=torch.float64, requires_grad=True)
    params = [torch.tensor(t, dtype=torch.float64) for W, b in layers for t in (W, b)]
    yt = O.torch_forward(xt, params)
    gt = torch.autograd.grad(yt, xt, torch.ones_like(yt) if u is None else torch.tensor(u, dtype=torch.float64))[0]
    assert np.max(np.abs(y.cpu().numpy() - yt.detach().numpy())) <= 1e-4
    assert np.max(np.abs(g.cpu().numpy() - gt.numpy())) <= tol_rel(gt.numpy())
    y1, g1_ = eng.forward_grad(ws, xd, ud if weighted else None)
    assert torch.allclose(y, y1, rtol=0, atol=2e-5) and torch.allclose(g, g1_, rtol=0, atol=2e-5 * max(1., float(g1_.abs().max())))
