"""Host-side checks that need no GPU: the C ABI library loads and exports every symbol include/siren_amd.h
declares, host-only ABI queries, module API / parameter names / init parity with the reference, the product
path refusing CPU tensors, get_mgrid."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, 'include', 'siren_amd.h')).read()
    return sorted(set(re.findall(r'^\s*(?:int32_t|const char\*)\s+(siren_\w+)\s*\(', src, re.M)))


@pytest.fixture(scope='module')
def lib():
    import __graft_entry__
    __graft_entry__.build()
    from siren_amd import _lib
    return _lib.load()


def test_library_exports_every_header_symbol(lib):
    names = header_functions()
    assert len(names) >= 9, names
    for n in names:
        assert hasattr(lib, n), n
    from siren_amd import _lib
    assert set(names) == set(_lib.EXPORTED)


def test_library_is_gfx950_code_object():
    import subprocess
    so = os.path.join(ROOT, 'siren_amd', 'libsiren_amd.so')
    out = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-readelf', '-S', so], capture_output=True, text=True).stdout
    assert '.hip_fatbin' in out


def test_param_count_and_workspace(lib):
    from siren_amd import _lib
    cfg = _lib.SirenCfg(2, 256, 3, 1, 30., 30., 1, 0)
    c = ctypes.c_int64()
    assert lib.siren_param_count(ctypes.byref(cfg), ctypes.byref(c)) == 0 and c.value == 198401
    assert lib.siren_workspace_floats(ctypes.byref(cfg), ctypes.byref(c)) == 0
    assert c.value == 2 * (4096 + 2 * 3 * 16 * 4096)  # unscaled image + the W1 kernel's phase-scaled copy
    assert lib.siren_train_ws_floats(ctypes.byref(cfg), 1000, ctypes.byref(c)) == 0 and c.value > 0
    bad = _lib.SirenCfg(2, 100, 3, 1, 30., 30., 1, 0)   # not a multiple of 64: no kernel path
    assert lib.siren_workspace_floats(ctypes.byref(bad), ctypes.byref(c)) == _lib.SIREN_EUNSUPPORTED
    assert b'256' in lib.siren_last_error()
    # hidden 1024 (train_video.py's width): the layered path; ws = the parameters + W_l^T only (immutable, ABI 5)
    big = _lib.SirenCfg(3, 1024, 3, 3, 30., 30., 1, 0)
    assert lib.siren_param_count(ctypes.byref(big), ctypes.byref(c)) == 0
    P = c.value
    assert lib.siren_workspace_floats(ctypes.byref(big), ctypes.byref(c)) == 0
    assert c.value == (P + 63) // 64 * 64 + 3 * 1024 * 1024
    # the caller's chunk scratch: [u x 2] chunks of 16384 x 1024 + column-sum slabs (4 bias + 3 dWout + 3 dW0
    # matrices of 256 rows x 1024, dbout 256 x 3) + [a_l, cos_l x 4 layers] chunks unless the split stores them
    slabs = 2 * 16384 * 1024 + (4 + 3 + 3) * 256 * 1024 + 256 * 3
    for q in ('siren_forward_ws_floats', 'siren_forward_grad_ws_floats', 'siren_train_ws_floats'):
        assert getattr(lib, q)(ctypes.byref(big), 100000, ctypes.byref(c)) == 0
        assert c.value == slabs + 2 * 4 * 16384 * 1024, q
    # the stored split keeps a_l / cos_l of every layer over all n rows, then the chunk scratch without them
    # (n = 1000 < one chunk: chunk 1024 rows, 16 slab rows)
    assert lib.siren_train_stored_ws_floats(ctypes.byref(big), 1000, ctypes.byref(c)) == 0
    assert c.value == 2 * 4 * 1000 * 1024 + 2 * 1024 * 1024 + (4 + 3 + 3) * 16 * 1024 + 16 * 3
    fs = _lib.SirenCfg(3, 1024, 3, 3, 30., 30., 0, 0)   # final sine: not on the layered path
    assert lib.siren_workspace_floats(ctypes.byref(fs), ctypes.byref(c)) == _lib.SIREN_EUNSUPPORTED
    assert lib.siren_second_order_ws_floats(ctypes.byref(big), 10, 1, ctypes.byref(c)) == _lib.SIREN_EUNSUPPORTED
    assert lib.siren_param_count(None, ctypes.byref(c)) == _lib.SIREN_EINVAL
    wide = _lib.SirenCfg(3, 512, 3, 3, 30., 30., 1, 0)
    assert lib.siren_param_count(ctypes.byref(wide), ctypes.byref(c)) == 0 and c.value == 791555
    assert lib.siren_workspace_floats(ctypes.byref(wide), ctypes.byref(c)) == 0
    assert c.value == 7168 + 2 * 3 * 32 * 8192          # small block padded to 1 KiB + 32 KiB slices
    # hidden 512 second order (the two-stream jet): a-, zb-, z-jets of 4 layers over 2 x 32 columns + slabs
    assert lib.siren_second_order_ws_floats(ctypes.byref(wide), 10, 1, ctypes.byref(c)) == 0
    assert c.value > 3 * 4 * 64 * 512


def test_zero_coords_is_a_noop(lib):
    from siren_amd import _lib
    cfg = _lib.SirenCfg(2, 256, 3, 1, 30., 30., 1, 0)
    assert lib.siren_forward(ctypes.byref(cfg), None, None, 0, None, None) == 0
    assert lib.siren_forward(ctypes.byref(cfg), None, None, -1, None, None) == _lib.SIREN_EINVAL


def test_entry_points_reject_null_cfg(lib):
    """Every cfg-taking entry point in include/siren_amd.h validates cfg before reading it or touching the device:
    a NULL cfg is SIREN_EINVAL, never a crash (siren_second_order_batched_ws_floats used to dereference it first).
    No GPU is needed: the call must return before any HIP call."""
    from siren_amd import _lib
    hdr = open(os.path.join(ROOT, 'include', 'siren_amd.h')).read()
    names = re.findall(r'^int32_t (siren_\w+)\(const siren_cfg\* cfg', hdr, re.M)
    assert 'siren_second_order_batched_ws_floats' in names and len(names) >= 30
    for name in names:
        assert name in _lib._SIGS and _lib._SIGS[name][0] is _lib._CFG, name
        c = _lib._I64(-7)
        args = []
        for t in _lib._SIGS[name]:
            if t is _lib._CFG or t is _lib._P:
                args.append(None)
            elif t is ctypes.POINTER(_lib._I64):
                args.append(ctypes.byref(c))
            else:
                args.append(t(16) if t is _lib._I64 else t(1))
        assert getattr(lib, name)(*args) == _lib.SIREN_EINVAL, name
        assert c.value == -7, name   # the count is left untouched on failure
        assert lib.siren_last_error(), name


def test_state_dict_keys_and_seed0_init_match_reference(g1, manifest):
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(0)
    m = SingleBVPNet(type='sine', in_features=2, out_features=1, verbose=False)
    sd = m.state_dict()
    assert list(sd.keys()) == manifest['state_dict_keys_5x256_d2']
    for k, v in sd.items():
        assert np.array_equal(v.numpy(), g1['w_' + k]), k   # bit-identical RNG replay of the reference init


def test_g4_init_matches(g4):
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(0)
    m = SingleBVPNet(out_features=3, in_features=3, hidden_features=512, num_hidden_layers=3, verbose=False)
    for k, v in m.state_dict().items():
        assert np.array_equal(v.numpy(), g4['w_' + k]), k


def test_cpu_tensors_are_refused():
    from siren_amd.modules import SingleBVPNet
    m = SingleBVPNet(verbose=False)
    with pytest.raises(RuntimeError, match='ROCm'):
        m({'coords': torch.zeros(1, 10, 2)})


def test_unsupported_modes_raise():
    from siren_amd.modules import SingleBVPNet
    from siren_amd._lib import SirenUnsupported
    with pytest.raises(SirenUnsupported):
        SingleBVPNet(mode='nerf', verbose=False)


def test_notebook_siren_api():
    from siren_amd.modules import Siren, SineLayer
    torch.manual_seed(0)
    s = Siren(2, 64, 2, 1, outermost_linear=True, first_omega_0=30, hidden_omega_0=30.)
    keys = list(s.state_dict().keys())
    assert keys[0] == 'net.0.linear.weight' and keys[-1] == 'net.3.bias'
    assert isinstance(s.net[0], SineLayer) and s.net[0].is_first
    assert float(s.net[0].linear.weight.detach().abs().max()) <= 0.5


def test_relu_baseline_runs_on_cpu():
    """Non-sine baselines keep the reference's plain torch layers (not the SIREN hot path)."""
    from siren_amd.modules import SingleBVPNet
    m = SingleBVPNet(type='relu', verbose=False)
    out = m({'coords': torch.rand(1, 5, 2)})
    assert out['model_out'].shape == (1, 5, 1) and out['model_in'].requires_grad


def test_get_subdict():
    from collections import OrderedDict
    from siren_amd.modules import get_subdict
    d = OrderedDict([('net.0.weight', 1), ('net.0.bias', 2), ('net.10.weight', 3), ('other', 4)])
    assert get_subdict(d, 'net.0') == OrderedDict([('weight', 1), ('bias', 2)])
    assert get_subdict(d, None) is d and get_subdict(None, 'x') is None


def test_get_mgrid_matches_reference_formula():
    from siren_amd.dataio import get_mgrid
    g = get_mgrid(256)
    assert g.shape == (65536, 2) and g.dtype == torch.float32
    assert torch.allclose(g[1], torch.tensor([-1., -0.99215686]))
    assert float(g.min()) == -1. and float(g.max()) == 1.
    g3 = get_mgrid((1, 4, 5), 3)
    assert g3.shape == (20, 3) and float(g3[:, 0].max()) == -1.   # dim 0 divides by max(s0 - 1, 1)


def test_hypernetwork_predicts_reference_weights(g7):
    """siren_amd.meta_modules.HyperNetwork (meta_modules.py:10-53, 136-154) built under the reference's seed
    predicts the reference's hypo-network weights exactly (same RNG consumption, plain torch on the CPU)."""
    import torch
    from siren_amd.meta_modules import HyperNetwork
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(8)
    hypo = SingleBVPNet(in_features=2, out_features=1, verbose=False)
    hyper = HyperNetwork(hyper_in_features=8, hyper_hidden_layers=1, hyper_hidden_features=32, hypo_module=hypo)
    z = torch.randn(3, 8)
    with torch.no_grad():
        params = hyper(z)
    assert list(params.keys()) == ['net.net.%d.0.%s' % (i, k) for i in range(5) for k in ('weight', 'bias')]
    for k, v in params.items():
        assert np.array_equal(v.numpy(), g7['p_' + k]), k


def test_new_entry_points_validate_before_any_device_work(lib):
    """Argument validation of the split / batched / per-step entry points happens on the host (no HIP call):
    NULL buffers, negative sizes and unsupported networks come back as status codes with siren_last_error text."""
    from siren_amd import _lib
    P = ctypes.c_void_p
    cfg = _lib.SirenCfg(2, 256, 3, 1, 30., 30., 1, 0)
    cnt = ctypes.c_int64()
    assert lib.siren_train_stored_ws_floats(ctypes.byref(cfg), 1000, ctypes.byref(cnt)) == 0 and cnt.value > 0
    lin0 = _lib.SirenCfg(2, 256, 3, 1, 30., 30., 0, 0)  # notebook Siren with a final sine: no stored split
    assert lib.siren_train_stored_ws_floats(ctypes.byref(lin0), 10, ctypes.byref(cnt)) == _lib.SIREN_EUNSUPPORTED
    assert lib.siren_last_error()
    assert lib.siren_forward_store(ctypes.byref(cfg), None, None, 0, None, None, None) == 0
    assert lib.siren_forward_store(ctypes.byref(cfg), None, None, 5, None, None, None) == _lib.SIREN_EINVAL
    assert lib.siren_backward_stored(ctypes.byref(cfg), None, None, 5, None, None, None, None, None) == \
        _lib.SIREN_EINVAL
    assert lib.siren_forward_laplace_store(ctypes.byref(cfg), None, None, -1, None, None, None, None, None) == \
        _lib.SIREN_EINVAL
    assert lib.siren_second_order_kept(ctypes.byref(cfg), None, None, 5, None, None, None, None, None, None,
                                       None) == _lib.SIREN_EINVAL
    assert lib.siren_forward_batched(ctypes.byref(cfg), None, None, 10, 70000, None, None) == _lib.SIREN_EINVAL
    assert lib.siren_forward_batched(ctypes.byref(cfg), None, None, 10, 0, None, None) == 0
    assert lib.siren_pack_batched(ctypes.byref(cfg), None, 3, None, None) == _lib.SIREN_EINVAL
    assert lib.siren_sample_sdf(None, None, 0, 10, 0, 0, None, None, None, None) == _lib.SIREN_EINVAL
    assert lib.siren_sample_sdf(None, None, 5, 0, 0, 0, None, None, None, None) == 0
    assert lib.siren_adam_step(None, None, None, None, 10, 1e-3, .9, .999, 1e-8, 0, 0., None, None) == \
        _lib.SIREN_EINVAL  # step must be >= 1
    assert lib.siren_adam_step(P(4), P(16), P(16), P(16), 10, 1e-3, .9, .999, 1e-8, 1, 0., None, None) == \
        _lib.SIREN_EINVAL  # 16-byte alignment
    assert lib.siren_adam_scratch_floats(ctypes.byref(cnt)) == 0 and cnt.value > 1024
    wide = _lib.SirenCfg(3, 512, 3, 3, 30., 30., 1, 0)
    assert lib.siren_second_order_ex(ctypes.byref(wide), None, None, 1, None, None, None, None, None, None, None,
                                     None) == _lib.SIREN_EINVAL   # hidden 512 is covered; NULL buffers are not
    assert lib.siren_second_order_kept(ctypes.byref(wide), P(64), P(64), 1, P(64), None, P(64), P(64), P(64), None,
                                       None) == _lib.SIREN_EUNSUPPORTED  # the kept forward is hidden 256 only


def test_workspace_queries_at_zero_coords_and_caller_owned_scratch(lib):
    """Every workspace query answers for n = 0 (the split-K plans used to divide by a zero tile count), and the
    hidden-512 W1 takes its cos scratch from the caller (siren_forward_grad_ws_floats; no allocation inside the
    library, SURVEY.md §8b ownership)."""
    from siren_amd import _lib
    cnt = ctypes.c_int64()
    cfg = _lib.SirenCfg(2, 256, 3, 1, 30., 30., 1, 0)
    wide = _lib.SirenCfg(3, 512, 3, 3, 30., 30., 1, 0)
    for c in (cfg, wide):
        assert lib.siren_train_ws_floats(ctypes.byref(c), 0, ctypes.byref(cnt)) == 0
        assert lib.siren_train_stored_ws_floats(ctypes.byref(c), 0, ctypes.byref(cnt)) == 0
        assert lib.siren_forward_grad_ws_floats(ctypes.byref(c), 0, ctypes.byref(cnt)) == 0 and cnt.value == 0
    for q in ('siren_laplace_backward_ws_floats', 'siren_hvp_backward_ws_floats'):
        assert getattr(lib, q)(ctypes.byref(cfg), 0, ctypes.byref(cnt)) == 0
    assert lib.siren_second_order_ws_floats(ctypes.byref(cfg), 0, 1, ctypes.byref(cnt)) == 0
    assert lib.siren_forward_grad_ws_floats(ctypes.byref(cfg), 4096, ctypes.byref(cnt)) == 0 and cnt.value == 0
    assert lib.siren_forward_grad_ws_floats(ctypes.byref(wide), 4096, ctypes.byref(cnt)) == 0
    assert cnt.value == 3 * 4096 * 512
    # hidden 512 without the workspace: refused on the host, before any launch
    P = ctypes.c_void_p
    assert lib.siren_forward_grad(ctypes.byref(wide), P(64), P(64), 10, None, None, P(64), None, None) == \
        _lib.SIREN_EINVAL
    assert b'tws' in lib.siren_last_error()
    # the third-order adjoint validates like the others
    assert lib.siren_hvp_backward(ctypes.byref(cfg), None, None, 5, None, None, None, None, None, None, None, None,
                                  None) == _lib.SIREN_EINVAL
    assert lib.siren_hvp_backward_ws_floats(ctypes.byref(wide), 5, ctypes.byref(cnt)) == 0   # hidden 512: mixed jet
    fs = _lib.SirenCfg(2, 256, 3, 1, 30., 30., 0, 0)  # final sine: not covered
    assert lib.siren_hvp_backward_ws_floats(ctypes.byref(fs), 5, ctypes.byref(cnt)) == _lib.SIREN_EUNSUPPORTED


@pytest.mark.parametrize('key,args', [('mgrid_256', (256,)), ('mgrid_3x7', ((3, 7),)), ('mgrid_32_d3', (32, 3)),
                                      ('mgrid_16x32x48_d3', ((16, 32, 48), 3)), ('mgrid_1x4x5_d3', ((1, 4, 5), 3))])
def test_get_mgrid_bit_exact_vs_reference(g8, key, args):
    """siren_amd.dataio.get_mgrid == the reference's dataio.get_mgrid (dataio.py:20-40), bit for bit (G8 fixture,
    produced by importing the reference's dataio in the build container)."""
    from siren_amd.dataio import get_mgrid
    g = get_mgrid(*args)
    assert g.dtype == torch.float32 and np.array_equal(g.numpy(), g8[key])


@pytest.mark.parametrize('tag,args,kw,seed', [
    ('A', (2, 256, 3, 1), dict(outermost_linear=True), 0),
    ('B', (1, 256, 3, 1), dict(outermost_linear=True, first_omega_0=3000, hidden_omega_0=30.), 1),
    ('C', (2, 256, 3, 3), dict(outermost_linear=False), 2)])
def test_notebook_siren_init_matches_reference(g8, tag, args, kw, seed):
    """The notebook Siren (explore_siren.ipynb cell 3) built under the same seed has bit-identical weights (same
    RNG consumption: nn.Linear default init, then the SIREN uniform re-init), and the same state-dict keys."""
    from siren_amd.modules import Siren
    torch.manual_seed(seed)
    s = Siren(*args, **kw)
    sd = s.state_dict()
    ref = {k[len(tag) + 3:]: v for k, v in g8.items() if k.startswith(tag + '_w_')}
    assert list(sd.keys()) == list(ref.keys())
    for k, v in sd.items():
        assert np.array_equal(v.numpy(), ref[k]), k
