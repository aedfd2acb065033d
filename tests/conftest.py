import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (ROCm device) and libsiren_amd.so')
    config.addinivalue_line('markers', 'slow: long-running (still part of the default selection)')


def load_golden(name):
    path = os.path.join(GOLDEN, 'golden_%s.npz' % name)
    if not os.path.exists(path):
        # A missing fixture is a failure, never a skip: a push that drops a golden (e.g. a .gpurunignore edit)
        # must not turn the parity tests it pins into silent skips.
        pytest.fail('golden fixture %s missing (regenerate with tests/golden/make_golden.py in the build container)'
                    % name, pytrace=False)
    return dict(np.load(path))


@pytest.fixture(scope='session')
def g1():
    return load_golden('g1')


@pytest.fixture(scope='session')
def g2():
    return load_golden('g2')


@pytest.fixture(scope='session')
def g3():
    return load_golden('g3')


@pytest.fixture(scope='session')
def g4():
    return load_golden('g4')


@pytest.fixture(scope='session')
def manifest():
    import json
    with open(os.path.join(GOLDEN, 'manifest.json')) as f:
        return json.load(f)


@pytest.fixture(scope='session')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no ROCm device')
    import __graft_entry__
    __graft_entry__.build()
    return torch.device('cuda:0')


def torch_path_functions():
    """Every public function of siren_amd._torch_path (the device-torch recompute), enumerated from the module so a
    new fallback is covered without editing the guard."""
    import inspect
    from siren_amd import _torch_path
    return sorted(name for name, f in vars(_torch_path).items()
                  if not name.startswith('_') and inspect.isfunction(f) and f.__module__ == _torch_path.__name__)


def forbid_torch_path(monkeypatch, allow=()):
    """Make every device-torch recompute raise: a test that passes under it ran its derivatives on the HIP kernels."""
    from siren_amd import _torch_path
    for name in torch_path_functions():
        if name in allow:
            continue

        def boom(*a, _n=name, **k):
            raise AssertionError('device-torch recompute %s must not run' % _n)
        monkeypatch.setattr(_torch_path, name, boom)


@pytest.fixture
def no_torch_path(monkeypatch):
    """Fixture form of forbid_torch_path (every _torch_path function forbidden for the whole test)."""
    forbid_torch_path(monkeypatch)


def weights_of(fx):
    """Fixture weights as a flat fp32 vector in state_dict order, plus the (W, b) list."""
    from oracle import siren_oracle as O
    layers = O.layers_from_state(fx)
    return O.flatten(layers).astype(np.float32), layers


def g1_layers(fx):
    return weights_of(fx)[1]


@pytest.fixture(scope='session')
def g6():
    return load_golden('g6')


def pml_case(g6, tag):
    """(coords (1, n, d), gt dict, flat params, layers) of the G6 Helmholtz ('H') or wave ('W') case."""
    sub = {k[len(tag) + 1:]: v for k, v in g6.items() if k.startswith(tag + '_')}
    gt = {k[3:]: v for k, v in sub.items() if k.startswith('gt_')}
    flat, layers = weights_of(sub)
    return sub['coords'], gt, flat, layers


def pml_ref_grads(g6, tag):
    keys = ['net.net.%d.0.%s' % (i, k) for i in range(5) for k in ('weight', 'bias')]
    return np.concatenate([g6['%s_grad_%s' % (tag, k)].reshape(-1) for k in keys])


@pytest.fixture(scope='session')
def g7():
    return load_golden('g7')


@pytest.fixture(scope='session')
def g8():
    return load_golden('g8')


@pytest.fixture(scope='session')
def g9():
    return load_golden('g9')


@pytest.fixture(scope='session')
def g10():
    return load_golden('g10')


@pytest.fixture(scope='session')
def g11():
    return load_golden('g11')
