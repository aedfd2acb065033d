"""siren_amd — MI355X-native SIREN engine: the reference's SIREN modules on fused HIP/CDNA4 kernels.

Public surface (mirrors xvdp/siren): modules.SingleBVPNet / FCBlock / BatchLinear / Sine / SineLayer / Siren,
diff_operators.{gradient, divergence, laplace, jacobian, hessian}, loss_functions.{image_mse, gradients_mse,
laplace_mse, sdf}, dataio.get_mgrid, training.train, plus the engine (SirenEngine) over the C ABI in
include/siren_amd.h. libsiren_amd.so is required: there is no CPU fallback.
"""
from . import _lib
from .engine import SirenEngine

__all__ = ['SirenEngine', 'modules', 'diff_operators', 'loss_functions', 'dataio', 'training', 'distributed']
