"""ctypes binding of the C ABI in include/siren_amd.h (libsiren_amd.so, built in-tree by __graft_entry__.build()).

This is the "reference-side binding" of the drop-in boundary: the reference (xvdp/siren) is pure PyTorch, so
its FFI for this path is a Python module. Everything here is plain pointers and sizes; torch only supplies
device memory and the current HIP stream (see siren_amd/engine.py).

The library is REQUIRED: importing the engine without it raises, there is no CPU or eager fallback.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('SIREN_AMD_LIB', os.path.join(_HERE, 'libsiren_amd.so'))
ABI_VERSION = 7

# Error codes (include/siren_amd.h)
SIREN_OK, SIREN_EINVAL, SIREN_EUNSUPPORTED, SIREN_EHIP = 0, 1, 2, 3


class SirenCfg(ctypes.Structure):
    """struct siren_cfg (include/siren_amd.h)."""
    _fields_ = [('d_in', ctypes.c_int32), ('hidden', ctypes.c_int32), ('n_hidden', ctypes.c_int32),
                ('d_out', ctypes.c_int32), ('omega_first', ctypes.c_float), ('omega_hidden', ctypes.c_float),
                ('outermost_linear', ctypes.c_int32), ('reserved', ctypes.c_int32)]


class SirenUnsupported(RuntimeError):
    """A valid SIREN configuration that the fused kernels do not cover (SIREN_EUNSUPPORTED)."""


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_CFG = ctypes.POINTER(SirenCfg)

# name -> argtypes; every entry point returns int32 status
_SIGS = {
    'siren_param_count': [_CFG, ctypes.POINTER(_I64)],
    'siren_workspace_floats': [_CFG, ctypes.POINTER(_I64)],
    'siren_pack': [_CFG, _P, _P, _P],
    'siren_forward': [_CFG, _P, _P, _I64, _P, _P],
    'siren_forward_ws_floats': [_CFG, _I64, ctypes.POINTER(_I64)],
    'siren_forward_ex': [_CFG, _P, _P, _I64, _P, _P, _P],
    'siren_forward_grad_ws_floats': [_CFG, _I64, ctypes.POINTER(_I64)],
    'siren_forward_grad': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P],
    'siren_forward_laplace': [_CFG, _P, _P, _I64, _P, _P, _P, _P],
    'siren_train_ws_floats': [_CFG, _I64, ctypes.POINTER(_I64)],
    'siren_backward': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P, _P],
    'siren_laplace_backward_ws_floats': [_CFG, _I64, ctypes.POINTER(_I64)],
    'siren_laplace_backward': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P],
    'siren_second_order_ws_floats': [_CFG, _I64, ctypes.c_int32, ctypes.POINTER(_I64)],
    'siren_second_order': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P],
    'siren_second_order_seeded': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P, _P],
    'siren_train_stored_ws_floats': [_CFG, _I64, ctypes.POINTER(_I64)],
    'siren_forward_store': [_CFG, _P, _P, _I64, _P, _P, _P],
    'siren_backward_stored': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P],
    'siren_forward_grad_store': [_CFG, _P, _P, _I64, _P, _P, _P, _P],
    'siren_second_order_kept': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _P],
    'siren_forward_laplace_store': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P],
    'siren_laplace_backward_stored': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P],
    'siren_train_batched_ws_floats': [_CFG, _I64, _I64, ctypes.POINTER(_I64)],
    'siren_pack_batched': [_CFG, _P, _I64, _P, _P],
    'siren_forward_batched': [_CFG, _P, _P, _I64, _I64, _P, _P],
    'siren_forward_batched_ex': [_CFG, _P, _P, _I64, _I64, _P, _P, _P],
    'siren_forward_grad_batched': [_CFG, _P, _P, _I64, _I64, _P, _P, _P, _P, _P],
    'siren_backward_batched': [_CFG, _P, _P, _I64, _I64, _P, _P, _P, _P, _P],
    'siren_sample_sdf': [_P, _P, _I64, _I64, ctypes.c_uint64, ctypes.c_uint64, _P, _P, _P, _P],
    'siren_adam_scratch_floats': [ctypes.POINTER(_I64)],
    'siren_w3_phase_profile': [_P],
    'siren_mc_ws_bytes': [_I64, _I64, _I64, ctypes.POINTER(_I64)],
    'siren_mc_count': [_P, _I64, _I64, _I64, ctypes.c_float, _P, ctypes.POINTER(_I64), ctypes.POINTER(_I64), _P],
    'siren_mc_emit': [_P, _I64, _I64, _I64, ctypes.c_float, _P, _P, _P, _P, _P],
    'siren_adam_step': [_P, _P, _P, _P, _I64, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _I64,
                        ctypes.c_float, _P, _P],
    'siren_second_order_ex': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _P],
    'siren_train_stored_batched_ws_floats': [_CFG, _I64, _I64, ctypes.POINTER(_I64)],
    'siren_forward_store_batched': [_CFG, _P, _P, _I64, _I64, _P, _P, _P],
    'siren_backward_stored_batched': [_CFG, _P, _P, _I64, _I64, _P, _P, _P, _P, _P],
    'siren_hvp_backward_ws_floats': [_CFG, _I64, ctypes.POINTER(_I64)],
    'siren_hvp_backward': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    'siren_w1_phase_profile': [_CFG, _P, _P, _I64, _P, _P, _P, _P],
    'siren_split_ws_floats': [_CFG, ctypes.POINTER(_I64)],
    'siren_pack_split': [_CFG, _P, _P, _P],
    'siren_forward_grad_split': [_CFG, _P, _P, _I64, _P, _P, _P],
    'siren_forward_split': [_CFG, _P, _P, _I64, _P, _P],
    'siren_backward_split': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P],
    'siren_train_split_ws_floats': [_CFG, _I64, ctypes.POINTER(_I64)],
    'siren_forward_store_split': [_CFG, _P, _P, _I64, _P, _P, _P],
    'siren_backward_stored_split': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P],
    'siren_hessian_backward_ws_floats': [_CFG, _I64, ctypes.POINTER(_I64)],
    'siren_hessian_backward': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _P],
    'siren_hessian_ws_floats': [_CFG, _I64, ctypes.c_int32, ctypes.POINTER(_I64)],
    'siren_hessian': [_CFG, _P, _P, _I64, _P, _P, _P, _P],
    'siren_hessian_ex': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P, _P],
    'siren_hessian_backward_kept': [_CFG, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _P],
    'siren_pack_batched_ex': [_CFG, _P, _I64, _P, ctypes.c_int32, _P],
    'siren_second_order_batched_ws_floats': [_CFG, _I64, _I64, ctypes.c_int32, ctypes.POINTER(_I64)],
    'siren_second_order_batched': [_CFG, _P, _P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P],
    'siren_hvp_backward_batched_ws_floats': [_CFG, _I64, _I64, ctypes.POINTER(_I64)],
    'siren_hvp_backward_batched': [_CFG, _P, _P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P],
}
EXPORTED = ('siren_abi_version', 'siren_last_error') + tuple(_SIGS)

_lib = None


def load():
    """Load libsiren_amd.so once; raise ImportError (loudly) when it is missing or stale."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError('siren_amd: %s not found - build it with `python -c "import __graft_entry__ as g; '
                          'g.build()"` (hipcc --offload-arch=gfx950). There is no CPU fallback.' % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    lib.siren_abi_version.restype = ctypes.c_int32
    lib.siren_abi_version.argtypes = []
    lib.siren_last_error.restype = ctypes.c_char_p
    lib.siren_last_error.argtypes = []
    if lib.siren_abi_version() != ABI_VERSION:
        raise ImportError('siren_amd: ABI version mismatch (lib %d, python %d); rebuild'
                          % (lib.siren_abi_version(), ABI_VERSION))
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = ctypes.c_int32
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what):
    if rc == SIREN_OK:
        return
    msg = '%s failed (%d): %s' % (what, rc, load().siren_last_error().decode(errors='replace'))
    if rc == SIREN_EUNSUPPORTED:
        raise SirenUnsupported(msg)
    if rc == SIREN_EINVAL:
        raise ValueError(msg)
    raise RuntimeError(msg)
