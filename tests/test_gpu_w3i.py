"""The interleaved second-order adjoint (w3i_kernel.hpp, the default W3 since round 3) against the phase-serial
w3_kernel it replaces (SIREN_FLAG_W3_SERIAL): the same arithmetic in the same order, so gx, ydot and every
workspace output the weight gradients are built from agree BITWISE — for every (L, d, o), with and without the
theta part, the first-order seed gy, the output weighting u, ydot, the kept stored forward, ragged n and the
grouped (batched-weights) launch. The fp64 bar of the W3 path itself (reference goldens, torch fp64 autograd) is held
by tests/test_gpu_parity.py, test_gpu_vector.py and test_gpu_batched.py, which now run on this kernel."""
import numpy as np
import pytest
import torch

from test_gpu_parity import random_layers, to_dev, torch_second_order_ref, tol_rel
from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu

SERIAL = 4  # SIREN_FLAG_W3_SERIAL


def engines(d, L, o):
    from siren_amd.engine import SirenEngine
    return SirenEngine(d, 256, L, o), SirenEngine(d, 256, L, o, flags=SERIAL)


def inputs(n, d, o, seed, cuda):
    rng = np.random.default_rng(seed)
    x = to_dev(rng.uniform(-1, 1, (n, d)), cuda)
    v = to_dev(rng.normal(size=(n, d)), cuda)
    gy = to_dev(rng.normal(size=(n, o)), cuda)
    u = to_dev(rng.normal(size=(n, o)), cuda)
    return x, v, gy, u


def same(a, b, what):
    assert a.shape == b.shape, what
    assert torch.equal(a, b), '%s: max |diff| %g' % (what, float((a - b).abs().max()))


@pytest.mark.parametrize('L', [1, 2, 3])
@pytest.mark.parametrize('d,o', [(1, 1), (2, 1), (3, 1), (4, 1), (2, 3), (3, 4)])
def test_w3i_bitwise_vs_serial(cuda, L, d, o):
    n = 4097 + 13 * L + d
    layers = random_layers(d, L, o, seed=100 * L + 10 * d + o)
    ei, es = engines(d, L, o)
    flat = to_dev(O.flatten(layers), cuda)
    wi, wsr = ei.pack(flat), es.pack(flat)
    x, v, gy, u = inputs(n, d, o, L + d + o, cuda)
    for theta in (False, True):
        for kw in ({}, {'gy': gy}, {'u': u, 'want_ydot': True}, {'gy': gy, 'u': u, 'want_ydot': True}):
            ri = ei.second_order(wi, x, v, want_theta=theta, **kw)
            rs = es.second_order(wsr, x, v, want_theta=theta, **kw)
            for k, (a, b) in enumerate(zip(ri, rs)):
                if a is None:
                    assert b is None
                    continue
                same(a, b, 'L%d d%d o%d theta %s %s output %d' % (L, d, o, theta, sorted(kw), k))


@pytest.mark.parametrize('n', [1, 15, 64, 65, 1000])
def test_w3i_ragged_and_kept(cuda, n):
    d, L, o = 3, 3, 1
    layers = random_layers(d, L, o, seed=n)
    ei, es = engines(d, L, o)
    flat = to_dev(O.flatten(layers), cuda)
    wi, wsr = ei.pack(flat), es.pack(flat)
    x, v, gy, _ = inputs(n, d, o, n, cuda)
    _, _, kept = ei.forward_grad_store(wi, x)
    for theta in (False, True):
        for kk in (None, kept):
            ri = ei.second_order(wi, x, v, want_theta=theta, gy=gy, kept=kk)
            rs = es.second_order(wsr, x, v, want_theta=theta, gy=gy, kept=kk)
            same(ri[0], rs[0], 'gx n=%d theta %s kept %s' % (n, theta, kk is not None))
            if theta:
                same(ri[1], rs[1], 'gtheta n=%d kept %s' % (n, kk is not None))


def test_w3i_vs_fp64(cuda):
    """The interleaved kernel against torch fp64 autograd (H v and the mixed theta gradient), 5x256, d 2."""
    n, d, L = 3000, 2, 3
    layers = random_layers(d, L, 1, seed=5)
    ei, _ = engines(d, L, 1)
    ws = ei.pack(to_dev(O.flatten(layers), cuda))
    rng = np.random.default_rng(9)
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    v = rng.normal(size=(n, d)).astype(np.float32)
    gx, gp = ei.second_order(ws, to_dev(x, cuda), to_dev(v, cuda))
    rgx, rgp = torch_second_order_ref(x, layers, v)
    assert np.max(np.abs(gx.cpu().numpy() - rgx)) <= tol_rel(rgx)
    assert np.max(np.abs(gp.cpu().numpy() - rgp)) <= 1e-4 * np.max(np.abs(rgp))


@pytest.mark.parametrize('L,B,n', [(1, 5, 777), (3, 5, 777), (3, 3, 512), (2, 2, 64), (3, 4, 100)])
def test_w3i_grouped_bitwise(cuda, L, B, n):
    """The grouped launch over batched weights (siren_second_order_batched, grid.y = element), with and without the
    output weighting u, the seed gy and ydot (the batched HVP node's forward is want_theta=False with u)."""
    d, o = 2, 1
    ei, es = engines(d, L, o)
    flats = torch.stack([to_dev(O.flatten(random_layers(d, L, o, seed=40 + b)), cuda) for b in range(B)])
    wi, wsr = ei.pack_batched(flats, full=True), es.pack_batched(flats, full=True)
    rng = np.random.default_rng(L + n)
    x = to_dev(rng.uniform(-1, 1, (B, n, d)), cuda)
    v = to_dev(rng.normal(size=(B, n, d)), cuda)
    u = to_dev(rng.normal(size=(B, n, o)), cuda)
    gy = to_dev(rng.normal(size=(B, n, o)), cuda)
    for theta in (False, True):
        for kw in ({}, {'u': u}, {'gy': gy, 'u': u, 'want_ydot': True}):
            ri = ei.second_order_batched(wi, x, v, want_theta=theta, **kw)
            rs = es.second_order_batched(wsr, x, v, want_theta=theta, **kw)
            for k, (a, b) in enumerate(zip(ri, rs)):
                if a is not None:
                    same(a, b, 'grouped L%d B%d n%d theta %s %s output %d' % (L, B, n, theta, sorted(kw), k))
