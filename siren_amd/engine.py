"""SirenEngine: torch-side plumbing around the C ABI (include/siren_amd.h).

torch supplies device memory (caching allocator) and the current HIP stream; every byte of SIREN arithmetic
runs in libsiren_amd.so. Inputs are validated here (shape / dtype / device) before any pointer crosses the ABI,
mirroring the reference's behaviour of raising on bad inputs (a torch shape error in BatchLinear.forward,
modules.py:23).
"""
import ctypes

import torch

from . import _lib

_ALIGN = 64  # the fused kernels process coordinates in tiles of 64 (TILE in siren_common.h)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class SirenEngine:
    """One SIREN architecture (d_in -> H x (n_hidden+1) -> d_out, sine activations) on the HIP kernels.

    Parameters follow SingleBVPNet / FCBlock (modules.py:37-160) and the notebook Siren (ipynb:110-166).
    """

    def __init__(self, d_in, hidden, n_hidden, d_out, omega_first=30., omega_hidden=30., outermost_linear=True,
                 flags=0):
        self.lib = _lib.load()
        self.cfg = _lib.SirenCfg(int(d_in), int(hidden), int(n_hidden), int(d_out), float(omega_first),
                                 float(omega_hidden), 1 if outermost_linear else 0, int(flags))
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_param_count(ctypes.byref(self.cfg), ctypes.byref(cnt)), 'siren_param_count')
        self.param_count = cnt.value
        rc = self.lib.siren_workspace_floats(ctypes.byref(self.cfg), ctypes.byref(cnt))
        self.supported = rc == _lib.SIREN_OK
        self.unsupported_reason = None if self.supported else self.lib.siren_last_error().decode()
        self.ws_floats = cnt.value if self.supported else 0
        # hidden 256 keeps cos(w z_l) of every layer in registers (1..3 hidden layers); hidden 512 spills it; other
        # widths run the layered path (layered.hip: rocBLAS layer GEMMs + fused epilogues, W0 / W1 / W2 only)
        self.layered = int(hidden) not in (256, 512)
        # hidden 256 at 4..5 hidden layers: cos no longer fits the registers, so W1 / W2 / the kept W3 run the stored
        # split through HBM (siren_capi.hip deep(): MODE_FWDS + MODE_REV) and W3 the serial kernel
        self.deep = (int(hidden) == 256 and 4 <= n_hidden <= 5 and bool(outermost_linear) and omega_first != 0
                     and omega_hidden != 0 and not (int(flags) & 1))
        self.grad_supported = self.supported and (1 <= n_hidden <= 3 or int(hidden) == 512 or self.layered
                                                  or self.deep)
        # the W3 second-order kernel: hidden 256, d_out <= 4 (vector outputs via an output weighting), linear output
        # the W4 jet kernel (fused Laplacian): hidden 256, d_in <= 2, linear output, 1..5 hidden layers
        self.laplace_supported = (self.supported and int(hidden) == 256 and int(d_in) <= 2 and 1 <= n_hidden <= 5
                                  and bool(outermost_linear) and omega_first != 0 and omega_hidden != 0)
        # stored-forward W2 split: training forward keeps a_l / cos, backward is reverse-only
        # (layered widths: a_l / cos_l of every layer over all n rows, see stored_for)
        self.stored_supported = (self.supported and bool(outermost_linear) and not (int(flags) & 1) and
                                 (int(hidden) == 512 or self.layered or (1 <= n_hidden <= 5 and omega_first != 0
                                                                         and omega_hidden != 0)))
        # hidden 512: the two-stream jet kernel (wide_jet_kernel.hpp), 1..8 hidden layers
        self.second_order_supported = (self.supported and int(d_out) <= 4 and bool(outermost_linear)
                                       and ((int(hidden) == 256 and (1 <= n_hidden <= 3 or self.deep))
                                            or int(hidden) == 512))
        # the third-order adjoint (mixed jet, siren_hvp_backward): linear output, hidden 256 with 1..5 hidden layers
        # or hidden 512 (wide_jet_kernel<4>)
        self.hvp_backward_supported = (self.supported and bool(outermost_linear)
                                       and ((int(hidden) == 256 and 1 <= n_hidden <= 5) or int(hidden) == 512))

    # the layered path's stored split keeps 2 (L + 1) n H floats; above this it recomputes the forward per chunk
    STORED_LAYERED_MAX_BYTES = 64 << 30

    def stored_for(self, n, batch=1):
        """Whether a training forward over n coordinates (x batch elements) keeps its activations for the backward."""
        if not self.stored_supported:
            return False
        if not self.layered:
            return True
        return 8 * (self.cfg.n_hidden + 1) * int(n) * self.cfg.hidden * int(batch) <= self.STORED_LAYERED_MAX_BYTES

    # ------------------------------------------------------------------------------------------------------
    def _require(self):
        if not self.supported:
            raise _lib.SirenUnsupported('siren_amd fused kernels do not cover this network: %s'
                                        % self.unsupported_reason)

    def _check_x(self, x):
        if not isinstance(x, torch.Tensor):
            raise TypeError('coords must be a torch.Tensor')
        if x.device.type != 'cuda':
            raise RuntimeError('siren_amd runs on ROCm devices (MI355X) only; got a %s tensor. The CPU restatement '
                               'of the reference lives in oracle/ and is test infrastructure.' % x.device.type)
        if x.dtype != torch.float32:
            raise TypeError('siren_amd computes in fp32; got %s' % x.dtype)
        if x.dim() != 2 or x.shape[1] != self.cfg.d_in:
            raise ValueError('coords must be (n, %d); got %s' % (self.cfg.d_in, tuple(x.shape)))
        return x.contiguous()

    def _check_params(self, flat, device):
        if flat.dtype != torch.float32 or flat.dim() != 1 or flat.numel() != self.param_count:
            raise ValueError('flat params must be fp32 with %d values; got %s %s'
                             % (self.param_count, flat.dtype, tuple(flat.shape)))
        if flat.device != device:
            raise ValueError('params on %s but coords on %s' % (flat.device, device))
        return flat.contiguous()

    # ------------------------------------------------------------------------------------------------------
    def pack(self, flat):
        """Repack the flat parameter vector into the kernels' slice layout (one small kernel launch)."""
        self._require()
        if flat.device.type != 'cuda':
            raise RuntimeError('siren_amd: parameters must live on a ROCm device')
        flat = self._check_params(flat, flat.device)
        ws = torch.empty(self.ws_floats, dtype=torch.float32, device=flat.device)
        _lib.check(self.lib.siren_pack(ctypes.byref(self.cfg), _ptr(flat), _ptr(ws), _stream(flat.device)),
                   'siren_pack')
        return ws

    def forward(self, ws, x, out=None):
        """W0: y = Phi(x) for x (n, d_in) -> y (n, d_out)."""
        self._require()
        x = self._check_x(x)
        n = x.shape[0]
        y = out if out is not None else torch.empty(n, self.cfg.d_out, dtype=torch.float32, device=x.device)
        tws = self._fwd_workspace(n, x.device)
        _lib.check(self.lib.siren_forward_ex(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(y), _ptr(tws),
                                             _stream(x.device)), 'siren_forward_ex')
        return y

    def forward_grad(self, ws, x, gy=None, want_y=True, out_y=None, out_gx=None):
        """W1 in one launch: y = Phi(x) and gx = sum_j gy_j dPhi_j/dx (gy=None: ones, i.e. the gradient
        diff_operators.gradient returns, diff_operators.py:39-43)."""
        self._require()
        if not self.grad_supported:
            raise _lib.SirenUnsupported('siren_forward_grad needs 1 <= num_hidden_layers <= 5 at hidden 256')
        x = self._check_x(x)
        n = x.shape[0]
        if gy is not None:
            if gy.shape != (n, self.cfg.d_out) or gy.dtype != torch.float32 or gy.device != x.device:
                raise ValueError('gy must be fp32 (%d, %d) on %s' % (n, self.cfg.d_out, x.device))
            gy = gy.contiguous()
        y = None
        if want_y:
            y = out_y if out_y is not None else torch.empty(n, self.cfg.d_out, dtype=torch.float32, device=x.device)
        gx = out_gx if out_gx is not None else torch.empty(n, self.cfg.d_in, dtype=torch.float32, device=x.device)
        tws = self._fg_workspace(n, x.device)
        _lib.check(self.lib.siren_forward_grad(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(gy), _ptr(y),
                                               _ptr(gx), _ptr(tws), _stream(x.device)), 'siren_forward_grad')
        return y, gx

    # ---- split-bf16 W1 (precision mode "bf16x6", w1x_kernel.hpp) ----------------------------------------
    @property
    def split_supported(self):
        """Whether siren_forward_grad_split covers this network (hidden 256, 3 hidden layers, d_in 2 / 3, d_out 1,
        linear output)."""
        c = self.cfg
        return (self.supported and c.hidden == 256 and c.n_hidden == 3 and c.d_out == 1 and c.d_in in (2, 3)
                and bool(c.outermost_linear) and c.omega_first != 0 and c.omega_hidden != 0)

    def pack_split(self, flat):
        """The split-bf16 weight image (siren_pack_split) from the flat parameters: once per weight update."""
        self._require()
        if not self.split_supported:
            raise _lib.SirenUnsupported('the split-bf16 W1 covers hidden 256, 3 hidden layers, in_features 2 / 3, '
                                        'out_features 1, linear output')
        if flat.device.type != 'cuda':
            raise RuntimeError('siren_amd: parameters must live on a ROCm device')
        flat = self._check_params(flat, flat.device)
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_split_ws_floats(ctypes.byref(self.cfg), ctypes.byref(cnt)), 'siren_split_ws_floats')
        wsx = torch.empty(cnt.value, dtype=torch.float32, device=flat.device)
        _lib.check(self.lib.siren_pack_split(ctypes.byref(self.cfg), _ptr(flat), _ptr(wsx), _stream(flat.device)),
                   'siren_pack_split')
        return wsx

    def forward_grad_split(self, wsx, x, want_y=True, out_y=None, out_gx=None):
        """W1 with gy = ones (diff_operators.gradient) on the split-bf16 kernel: (y, gx) as forward_grad(ws, x)."""
        self._require()
        if not self.split_supported:
            raise _lib.SirenUnsupported('the split-bf16 W1 covers hidden 256, 3 hidden layers, in_features 2 / 3, '
                                        'out_features 1, linear output')
        x = self._check_x(x)
        n = x.shape[0]
        y = None
        if want_y:
            y = out_y if out_y is not None else torch.empty(n, 1, dtype=torch.float32, device=x.device)
        gx = out_gx if out_gx is not None else torch.empty(n, self.cfg.d_in, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_forward_grad_split(ctypes.byref(self.cfg), _ptr(wsx), _ptr(x), n, _ptr(y), _ptr(gx),
                                                     _stream(x.device)), 'siren_forward_grad_split')
        return y, gx

    def forward_split(self, wsx, x, out=None):
        """W0 (y = Phi(x)) on the split-bf16 forward kernel (siren_forward_split): dense evaluation."""
        self._require()
        if not self.split_supported:
            raise _lib.SirenUnsupported('the split-bf16 kernels cover hidden 256, 3 hidden layers, in_features 2 / 3, '
                                        'out_features 1, linear output')
        x = self._check_x(x)
        n = x.shape[0]
        y = out if out is not None else torch.empty(n, 1, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_forward_split(ctypes.byref(self.cfg), _ptr(wsx), _ptr(x), n, _ptr(y),
                                                _stream(x.device)), 'siren_forward_split')
        return y

    def backward_split(self, wsx, x, gy, want_gx=False):
        """Training backward of the bf16x6 leg (siren_backward_split): (gx or None, gparams) for y =
        forward_split(wsx, x) — the split-bf16 kernel recomputes the forward and runs the reverse from gy, the fp32
        MFMA wgrad reduces the tiles."""
        self._require()
        if not self.split_supported:
            raise _lib.SirenUnsupported('the split-bf16 kernels cover hidden 256, 3 hidden layers, in_features 2 / 3, '
                                        'out_features 1, linear output')
        x = self._check_x(x)
        n = x.shape[0]
        gy = gy.contiguous()
        if gy.shape != (n, 1) or gy.dtype != torch.float32 or gy.device != x.device:
            raise ValueError('gy must be fp32 (%d, 1) on the coords device; got %s' % (n, tuple(gy.shape)))
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_train_ws_floats(ctypes.byref(self.cfg), n, ctypes.byref(cnt)),
                   'siren_train_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        gx = torch.empty(n, self.cfg.d_in, dtype=torch.float32, device=x.device) if want_gx else None
        gp = torch.empty(self.param_count, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_backward_split(ctypes.byref(self.cfg), _ptr(wsx), _ptr(x), n, _ptr(gy), _ptr(tws),
                                                 _ptr(gx), _ptr(gp), _stream(x.device)), 'siren_backward_split')
        return gx, gp

    def forward_store_split(self, wsx, x):
        """Training forward of the bf16x6 leg (siren_forward_store_split): (y, tws) — y from the split-bf16 forward, tws
        its a_l tiles and cos(w z_l) for backward_stored_split."""
        self._require()
        if not self.split_supported:
            raise _lib.SirenUnsupported('the split-bf16 kernels cover hidden 256, 3 hidden layers, in_features 2 / 3, '
                                        'out_features 1, linear output')
        x = self._check_x(x)
        n = x.shape[0]
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_train_split_ws_floats(ctypes.byref(self.cfg), n, ctypes.byref(cnt)),
                   'siren_train_split_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        y = torch.empty(n, 1, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_forward_store_split(ctypes.byref(self.cfg), _ptr(wsx), _ptr(x), n, _ptr(y), _ptr(tws),
                                                      _stream(x.device)), 'siren_forward_store_split')
        return y, tws

    def backward_stored_split(self, wsx, x, gy, tws, want_gx=False):
        """Reverse-only backward of the bf16x6 leg from forward_store_split's tws: (gx or None, gparams)."""
        self._require()
        if not self.split_supported:
            raise _lib.SirenUnsupported('the split-bf16 kernels cover hidden 256, 3 hidden layers, in_features 2 / 3, '
                                        'out_features 1, linear output')
        x = self._check_x(x)
        n = x.shape[0]
        gy = gy.contiguous()
        if gy.shape != (n, 1) or gy.dtype != torch.float32 or gy.device != x.device:
            raise ValueError('gy must be fp32 (%d, 1) on the coords device; got %s' % (n, tuple(gy.shape)))
        # the C side cannot tell a workspace of another n (or forward_store's) from this one: its kernels would read
        # cos and write deltas / partials out of bounds
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_train_split_ws_floats(ctypes.byref(self.cfg), n, ctypes.byref(cnt)),
                   'siren_train_split_ws_floats')
        if (tws.dtype != torch.float32 or tws.device != x.device or not tws.is_contiguous()
                or tws.numel() != cnt.value):
            raise ValueError('tws must be the contiguous fp32 workspace forward_store_split made for these %d coords '
                             '(%d floats on %s); got %d %s floats on %s'
                             % (n, cnt.value, x.device, tws.numel(), tws.dtype, tws.device))
        gx = torch.empty(n, self.cfg.d_in, dtype=torch.float32, device=x.device) if want_gx else None
        gp = torch.empty(self.param_count, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_backward_stored_split(ctypes.byref(self.cfg), _ptr(wsx), _ptr(x), n, _ptr(gy),
                                                        _ptr(tws), _ptr(gx), _ptr(gp), _stream(x.device)),
                   'siren_backward_stored_split')
        return gx, gp

    def _fwd_workspace(self, n, device):
        """siren_forward_ex's caller-owned scratch (the layered path's chunk scratch; None elsewhere)."""
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_forward_ws_floats(ctypes.byref(self.cfg), n, ctypes.byref(cnt)),
                   'siren_forward_ws_floats')
        return torch.empty(cnt.value, dtype=torch.float32, device=device) if cnt.value > 0 else None

    def _fg_workspace(self, n, device):
        """siren_forward_grad's caller-owned scratch (hidden 512: the cos spill; hidden 256: none)."""
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_forward_grad_ws_floats(ctypes.byref(self.cfg), n, ctypes.byref(cnt)),
                   'siren_forward_grad_ws_floats')
        return torch.empty(cnt.value, dtype=torch.float32, device=device) if cnt.value > 0 else None

    def hvp_backward(self, ws, x, v, g, u=None, want_theta=True, want_v=False, want_u=False):
        """Third-order adjoint: the backward of the Hessian-vector-product node h = sum_j u_j H_j(x) v given its
        cotangent g (siren_hvp_backward). Returns (gx, gparams | None, gv | None, gu | None) = d/d(x, theta, v, u)
        of sum_c <g_c, h_c>."""
        self._require()
        if not self.hvp_backward_supported:
            raise _lib.SirenUnsupported('siren_hvp_backward covers a linear output, hidden 256 (1..5 hidden layers) '
                                        'or hidden 512')
        x = self._check_x(x)
        n, d, o = x.shape[0], self.cfg.d_in, self.cfg.d_out
        for name, t, w in (('v', v, d), ('g', g, d), ('u', u, o)):
            if t is not None and (t.numel() != n * w or t.dtype != torch.float32 or t.device != x.device):
                raise ValueError('%s must be fp32 with %d values on %s' % (name, n * w, x.device))
        v, g = v.contiguous(), g.contiguous()
        u = u.contiguous() if u is not None else None
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_hvp_backward_ws_floats(ctypes.byref(self.cfg), n, ctypes.byref(cnt)),
                   'siren_hvp_backward_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        gx = torch.empty(n, d, dtype=torch.float32, device=x.device)
        gp = torch.empty(self.param_count, dtype=torch.float32, device=x.device) if want_theta else None
        gv = torch.empty(n, d, dtype=torch.float32, device=x.device) if want_v else None
        gu = torch.empty(n, o, dtype=torch.float32, device=x.device) if want_u else None
        _lib.check(self.lib.siren_hvp_backward(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(v), _ptr(u), _ptr(g),
                                               _ptr(tws), _ptr(gx), _ptr(gp), _ptr(gv), _ptr(gu), _stream(x.device)),
                   'siren_hvp_backward')
        return gx, gp, gv, gu

    @property
    def hessian_backward_supported(self):
        """siren_hessian_backward covers this network: hidden 256, 1..5 hidden layers, d_in <= 2, linear output."""
        c = self.cfg
        return (self.supported and c.hidden == 256 and 1 <= c.n_hidden <= 5 and c.d_in <= 2
                and bool(c.outermost_linear))

    def hessian(self, ws, x, u=None, keep=False, want_yg=False):
        """Hm (n, d_in, d_in) = sum_j u_j H_j(x) (u (n, d_out), None = ones) in one forward-mode second-order jet
        sweep (siren_hessian). keep=True also returns the per-layer jets (n-proportional fp32 buffer) that
        hessian_backward(..., kept=) reads instead of recomputing its forward: (hm, kept). want_yg=True returns
        (hm, kept, y, g) with y = Phi(x) (n, d_out) and g = sum_j u_j dPhi_j/dx (n, d_in) from the same sweep
        (siren_hessian_ex; kept None unless keep)."""
        self._require()
        if not self.hessian_backward_supported:
            raise _lib.SirenUnsupported('siren_hessian covers hidden 256, 1..5 hidden layers, in_features <= 2, '
                                        'linear output')
        x = self._check_x(x)
        n, d, o = x.shape[0], self.cfg.d_in, self.cfg.d_out
        if u is not None and (u.numel() != n * o or u.dtype != torch.float32 or u.device != x.device):
            raise ValueError('u must be fp32 (%d, %d) on %s' % (n, o, x.device))
        u = u.contiguous() if u is not None else None
        hm = torch.empty(n, d, d, dtype=torch.float32, device=x.device)
        kept = None
        if keep:
            cnt = ctypes.c_int64()
            _lib.check(self.lib.siren_hessian_ws_floats(ctypes.byref(self.cfg), n, 1, ctypes.byref(cnt)),
                       'siren_hessian_ws_floats')
            kept = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        if want_yg:
            y = torch.empty(n, o, dtype=torch.float32, device=x.device)
            g = torch.empty(n, d, dtype=torch.float32, device=x.device)
            _lib.check(self.lib.siren_hessian_ex(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(u), _ptr(kept),
                                                 _ptr(hm), _ptr(y), _ptr(g), _stream(x.device)), 'siren_hessian_ex')
            return hm, kept, y, g
        _lib.check(self.lib.siren_hessian(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(u), _ptr(kept), _ptr(hm),
                                          _stream(x.device)), 'siren_hessian')
        return (hm, kept) if keep else hm

    def hessian_backward(self, ws, x, G, u=None, want_theta=True, want_u=False, kept=None):
        """The backward of the Hessian node: d/d(x, theta, u) of sum_c <G_c, Hm_c> (siren_hessian_backward; with
        kept = hessian(ws, x, u, keep=True)[1] of the same inputs, siren_hessian_backward_kept skips the forward
        GEMMs). Returns (gx, gparams | None, gu | None)."""
        self._require()
        if not self.hessian_backward_supported:
            raise _lib.SirenUnsupported('siren_hessian_backward covers hidden 256, 1..5 hidden layers, in_features '
                                        '<= 2, linear output')
        x = self._check_x(x)
        n, d, o = x.shape[0], self.cfg.d_in, self.cfg.d_out
        if G.numel() != n * d * d or G.dtype != torch.float32 or G.device != x.device:
            raise ValueError('G must be fp32 (%d, %d, %d) on %s' % (n, d, d, x.device))
        if u is not None and (u.numel() != n * o or u.dtype != torch.float32 or u.device != x.device):
            raise ValueError('u must be fp32 (%d, %d) on %s' % (n, o, x.device))
        G = G.contiguous()
        u = u.contiguous() if u is not None else None
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_hessian_backward_ws_floats(ctypes.byref(self.cfg), n, ctypes.byref(cnt)),
                   'siren_hessian_backward_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        gx = torch.empty(n, d, dtype=torch.float32, device=x.device)
        gp = torch.empty(self.param_count, dtype=torch.float32, device=x.device) if want_theta else None
        gu = torch.empty(n, o, dtype=torch.float32, device=x.device) if want_u else None
        if kept is not None:
            cnt = ctypes.c_int64()
            _lib.check(self.lib.siren_hessian_ws_floats(ctypes.byref(self.cfg), n, 1, ctypes.byref(cnt)),
                       'siren_hessian_ws_floats')
            if kept.numel() != cnt.value or kept.dtype != torch.float32 or kept.device != x.device:
                raise ValueError('kept must be the fp32 buffer of hessian(..., keep=True) for these %d points' % n)
        _lib.check(self.lib.siren_hessian_backward_kept(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(G), _ptr(u),
                                                        _ptr(kept), _ptr(tws), _ptr(gx), _ptr(gp), _ptr(gu),
                                                        _stream(x.device)), 'siren_hessian_backward_kept')
        return gx, gp, gu

    def forward_laplace(self, ws, x, want_y=False, want_gx=False):
        """W4 in one launch: (y | None, sum_j grad y_j | None, sum_j Laplacian y_j (n, 1)) — what
        diff_operators.gradient / laplace return (diff_operators.py:27-43)."""
        self._require()
        if not self.laplace_supported:
            raise _lib.SirenUnsupported('siren_forward_laplace covers hidden 256, in_features <= 2, linear output, '
                                        '1..5 hidden layers')
        x = self._check_x(x)
        n = x.shape[0]
        y = torch.empty(n, self.cfg.d_out, dtype=torch.float32, device=x.device) if want_y else None
        gx = torch.empty(n, self.cfg.d_in, dtype=torch.float32, device=x.device) if want_gx else None
        lap = torch.empty(n, 1, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_forward_laplace(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(y), _ptr(gx),
                                                  _ptr(lap), _stream(x.device)), 'siren_forward_laplace')
        return y, gx, lap

    def laplace_backward(self, ws, x, glap):
        """W4s: (gx, gparams) = d/d(x, theta) of sum_c glap_c Laplacian(x_c) — the backward of the fused
        Laplacian node (laplace_mse training)."""
        self._require()
        if not self.laplace_supported:
            raise _lib.SirenUnsupported('siren_laplace_backward covers hidden 256, in_features <= 2, linear output, '
                                        '1..5 hidden layers')
        x = self._check_x(x)
        n = x.shape[0]
        glap = glap.reshape(-1).contiguous()
        if glap.numel() != n or glap.dtype != torch.float32 or glap.device != x.device:
            raise ValueError('glap must be fp32 with %d values on %s' % (n, x.device))
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_laplace_backward_ws_floats(ctypes.byref(self.cfg), n, ctypes.byref(cnt)),
                   'siren_laplace_backward_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        gx = torch.empty(n, self.cfg.d_in, dtype=torch.float32, device=x.device)
        gp = torch.empty(self.param_count, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_laplace_backward(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(glap),
                                                   _ptr(tws), _ptr(gx), _ptr(gp), _stream(x.device)),
                   'siren_laplace_backward')
        return gx, gp

    def forward_laplace_store(self, ws, x, want_y=False):
        """Split W4 (laplace_mse training forward): the Laplacian (n, 1) + the jet stores, kept in a workspace for
        laplace_backward_stored. Returns (lap, tws), or (lap, tws, y) with want_y (y = Phi(x) from the same sweep)."""
        self._require()
        x = self._check_x(x)
        n = x.shape[0]
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_laplace_backward_ws_floats(ctypes.byref(self.cfg), n, ctypes.byref(cnt)),
                   'siren_laplace_backward_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        lap = torch.empty(n, 1, dtype=torch.float32, device=x.device)
        y = torch.empty(n, self.cfg.d_out, dtype=torch.float32, device=x.device) if want_y else None
        _lib.check(self.lib.siren_forward_laplace_store(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(y), None,
                                                        _ptr(lap), _ptr(tws), _stream(x.device)),
                   'siren_forward_laplace_store')
        return (lap, tws, y) if want_y else (lap, tws)

    def laplace_backward_stored(self, ws, x, glap, tws):
        """Split W4s: (gx, gparams) from forward_laplace_store's workspace (reverse-only jet sweep)."""
        self._require()
        x = self._check_x(x)
        n = x.shape[0]
        glap = glap.reshape(-1).contiguous()
        gx = torch.empty(n, self.cfg.d_in, dtype=torch.float32, device=x.device)
        gp = torch.empty(self.param_count, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_laplace_backward_stored(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(glap),
                                                          _ptr(tws), _ptr(gx), _ptr(gp), _stream(x.device)),
                   'siren_laplace_backward_stored')
        return gx, gp

    # ------------------------------------------------------------------------------------------------------
    def backward_params(self, ws, x, gy):
        """W2 backward: (gx, gparams) for one coordinate batch, gparams flat in parameter order.

        Three launches: the fused forward+reverse kernel in store mode (sin activations and deltas of every
        layer to HBM), the split-K MFMA weight-gradient kernel, and the deterministic partial-slab reduction.
        """
        self._require()
        if not self.grad_supported:
            raise _lib.SirenUnsupported('siren_backward needs 1 <= num_hidden_layers <= 5 at hidden 256')
        x = self._check_x(x)
        n = x.shape[0]
        gy = gy.contiguous()
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_train_ws_floats(ctypes.byref(self.cfg), n, ctypes.byref(cnt)),
                   'siren_train_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        gx = torch.empty(n, self.cfg.d_in, dtype=torch.float32, device=x.device)
        gp = torch.empty(self.param_count, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_backward(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(gy), _ptr(tws),
                                           ctypes.c_void_p(0), _ptr(gx), _ptr(gp), _stream(x.device)),
                   'siren_backward')
        return gx, gp

    # ---- batched (hypernetwork) weights: element b of (B, ...) tensors uses its own parameter row ------------
    def _check_xb(self, x):
        if not isinstance(x, torch.Tensor) or x.device.type != 'cuda' or x.dtype != torch.float32:
            raise RuntimeError('siren_amd batched coords must be fp32 on a ROCm device')
        if x.dim() != 3 or x.shape[2] != self.cfg.d_in:
            raise ValueError('batched coords must be (B, n, %d); got %s' % (self.cfg.d_in, tuple(x.shape)))
        return x.contiguous()

    def pack_batched(self, flat, full=False):
        """flat (B, param_count) -> packed workspaces (B, ws_floats), one grouped launch. full=False writes what the
        first-order batched entry points read (hidden 256: the phase-scaled half only); full=True the whole image
        of every element, which second_order_batched / hvp_backward_batched and single-network calls need."""
        self._require()
        if flat.dim() != 2 or flat.shape[1] != self.param_count or flat.dtype != torch.float32 \
                or flat.device.type != 'cuda':
            raise ValueError('batched params must be fp32 (B, %d) on a ROCm device' % self.param_count)
        flat = flat.contiguous()
        ws = torch.empty(flat.shape[0], self.ws_floats, dtype=torch.float32, device=flat.device)
        _lib.check(self.lib.siren_pack_batched_ex(ctypes.byref(self.cfg), _ptr(flat), flat.shape[0], _ptr(ws),
                                                  1 if full else 0, _stream(flat.device)), 'siren_pack_batched_ex')
        return ws

    def _check_batched_like(self, name, t, shape, device):
        if t is None:
            return None
        if tuple(t.shape) != tuple(shape) or t.dtype != torch.float32 or t.device != device:
            raise ValueError('%s must be fp32 %s on %s; got %s %s' % (name, tuple(shape), device, t.dtype,
                                                                    tuple(t.shape)))
        return t.contiguous()

    def second_order_batched(self, ws, x, v, want_theta=True, gy=None, u=None, want_ydot=False):
        """second_order for every element of batched weights (ws from pack_batched(full=True)): x, v (B, n, d_in),
        u / gy (B, n, d_out) nullable. Returns (gx (B, n, d_in), gparams (B, P) | None[, ydot (B, n, d_out)])."""
        self._require()
        if not self.second_order_supported:
            raise _lib.SirenUnsupported('siren_second_order covers d_out <= 4, linear output, hidden 256 with 1..5 '
                                        'hidden layers (nonzero omegas beyond 3) or hidden 512')
        x = self._check_xb(x)
        B, n, d, o = x.shape[0], x.shape[1], self.cfg.d_in, self.cfg.d_out
        v = self._check_batched_like('v', v, (B, n, d), x.device)
        gy = self._check_batched_like('gy', gy, (B, n, o), x.device)
        u = self._check_batched_like('u', u, (B, n, o), x.device)
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_second_order_batched_ws_floats(ctypes.byref(self.cfg), n, B, 1 if want_theta else 0,
                                                                 ctypes.byref(cnt)), 'siren_second_order_batched_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        gx = torch.empty(B, n, d, dtype=torch.float32, device=x.device)
        gp = torch.empty(B, self.param_count, dtype=torch.float32, device=x.device) if want_theta else None
        ydot = torch.empty(B, n, o, dtype=torch.float32, device=x.device) if want_ydot else None
        _lib.check(self.lib.siren_second_order_batched(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, B, _ptr(v), _ptr(u),
                                                       _ptr(gy), _ptr(tws), _ptr(gx), _ptr(gp), _ptr(ydot),
                                                       _stream(x.device)), 'siren_second_order_batched')
        return (gx, gp, ydot) if want_ydot else (gx, gp)

    def hvp_backward_batched(self, ws, x, v, g, u=None, want_theta=True, want_v=False, want_u=False):
        """hvp_backward for every element of batched weights (ws from pack_batched(full=True)). Returns
        (gx (B, n, d_in), gparams (B, P) | None, gv | None, gu | None)."""
        self._require()
        if not self.hvp_backward_supported:
            raise _lib.SirenUnsupported('siren_hvp_backward covers a linear output, hidden 256 (1..5 hidden layers) '
                                        'or hidden 512')
        x = self._check_xb(x)
        B, n, d, o = x.shape[0], x.shape[1], self.cfg.d_in, self.cfg.d_out
        v = self._check_batched_like('v', v, (B, n, d), x.device)
        g = self._check_batched_like('g', g, (B, n, d), x.device)
        u = self._check_batched_like('u', u, (B, n, o), x.device)
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_hvp_backward_batched_ws_floats(ctypes.byref(self.cfg), n, B, ctypes.byref(cnt)),
                   'siren_hvp_backward_batched_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        gx = torch.empty(B, n, d, dtype=torch.float32, device=x.device)
        gp = torch.empty(B, self.param_count, dtype=torch.float32, device=x.device) if want_theta else None
        gv = torch.empty(B, n, d, dtype=torch.float32, device=x.device) if want_v else None
        gu = torch.empty(B, n, o, dtype=torch.float32, device=x.device) if want_u else None
        _lib.check(self.lib.siren_hvp_backward_batched(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, B, _ptr(v), _ptr(u),
                                                       _ptr(g), _ptr(tws), _ptr(gx), _ptr(gp), _ptr(gv), _ptr(gu),
                                                       _stream(x.device)), 'siren_hvp_backward_batched')
        return gx, gp, gv, gu

    def forward_batched(self, ws, x):
        """W0 over (B, n, d_in) with per-element weights -> (B, n, d_out)."""
        self._require()
        x = self._check_xb(x)
        B, n = x.shape[:2]
        y = torch.empty(B, n, self.cfg.d_out, dtype=torch.float32, device=x.device)
        tws = self._fwd_workspace(n, x.device)
        _lib.check(self.lib.siren_forward_batched_ex(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, B, _ptr(y), _ptr(tws),
                                                     _stream(x.device)), 'siren_forward_batched_ex')
        return y

    def forward_grad_batched(self, ws, x, gy=None, want_y=True):
        """W1 over (B, n, d_in): (y | None, J^T gy) with per-element weights."""
        self._require()
        if not self.grad_supported:
            raise _lib.SirenUnsupported('siren_forward_grad needs 1 <= num_hidden_layers <= 5 at hidden 256')
        x = self._check_xb(x)
        B, n = x.shape[:2]
        if gy is not None:
            gy = gy.contiguous()
            if gy.shape != (B, n, self.cfg.d_out):
                raise ValueError('gy must be (%d, %d, %d)' % (B, n, self.cfg.d_out))
        y = torch.empty(B, n, self.cfg.d_out, dtype=torch.float32, device=x.device) if want_y else None
        gx = torch.empty_like(x)
        tws = self._fg_workspace(n, x.device)
        _lib.check(self.lib.siren_forward_grad_batched(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, B, _ptr(gy),
                                                       _ptr(y), _ptr(gx), _ptr(tws), _stream(x.device)),
                   'siren_forward_grad_batched')
        return y, gx

    def backward_params_batched(self, ws, x, gy):
        """W2 per element: (gx (B, n, d_in), gparams (B, param_count))."""
        self._require()
        if not self.grad_supported:
            raise _lib.SirenUnsupported('siren_backward needs 1 <= num_hidden_layers <= 5 at hidden 256')
        x = self._check_xb(x)
        B, n = x.shape[:2]
        gy = gy.contiguous()
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_train_batched_ws_floats(ctypes.byref(self.cfg), n, B, ctypes.byref(cnt)),
                   'siren_train_batched_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        gx = torch.empty_like(x)
        gp = torch.empty(B, self.param_count, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_backward_batched(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, B, _ptr(gy),
                                                   _ptr(tws), _ptr(gx), _ptr(gp), _stream(x.device)),
                   'siren_backward_batched')
        return gx, gp

    def forward_store_batched(self, ws, x):
        """Training forward over batched weights (stored-forward split): y (B, n, d_out) plus every element's a_l
        tiles and cos(w z_l) in a workspace returned with y (siren_forward_store_batched)."""
        self._require()
        x = self._check_xb(x)
        B, n = x.shape[:2]
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_train_stored_batched_ws_floats(ctypes.byref(self.cfg), n, B, ctypes.byref(cnt)),
                   'siren_train_stored_batched_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        y = torch.empty(B, n, self.cfg.d_out, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_forward_store_batched(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, B, _ptr(y),
                                                        _ptr(tws), _stream(x.device)), 'siren_forward_store_batched')
        return y, tws

    def backward_stored_batched(self, ws, x, gy, tws):
        """Reverse-only W2 over batched weights from forward_store_batched's workspace: (gx (B, n, d_in),
        gparams (B, param_count))."""
        self._require()
        x = self._check_xb(x)
        B, n = x.shape[:2]
        gy = gy.contiguous()
        gx = torch.empty_like(x)
        gp = torch.empty(B, self.param_count, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_backward_stored_batched(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, B, _ptr(gy),
                                                          _ptr(tws), _ptr(gx), _ptr(gp), _stream(x.device)),
                   'siren_backward_stored_batched')
        return gx, gp

    def forward_store(self, ws, x):
        """Training forward (stored-forward W2 split): y plus the a_l tiles and cos(w z_l) the reverse-only
        backward needs, kept in a workspace returned with y."""
        self._require()
        x = self._check_x(x)
        n = x.shape[0]
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_train_stored_ws_floats(ctypes.byref(self.cfg), n, ctypes.byref(cnt)),
                   'siren_train_stored_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        y = torch.empty(n, self.cfg.d_out, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_forward_store(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(y), _ptr(tws),
                                                _stream(x.device)), 'siren_forward_store')
        return y, tws

    def forward_grad_store(self, ws, x):
        """Stored jet forward (hidden 256): (y, J = dPhi/dx, tws) with a_l / cos kept in tws for second_order(kept=)."""
        self._require()
        x = self._check_x(x)
        n = x.shape[0]
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_train_stored_ws_floats(ctypes.byref(self.cfg), n, ctypes.byref(cnt)),
                   'siren_train_stored_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        y = torch.empty(n, self.cfg.d_out, dtype=torch.float32, device=x.device)
        gx = torch.empty(n, self.cfg.d_in, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_forward_grad_store(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(y), _ptr(gx),
                                                     _ptr(tws), _stream(x.device)), 'siren_forward_grad_store')
        return y, gx, tws

    def backward_stored(self, ws, x, gy, tws):
        """W2 backward from forward_store's workspace: reverse sweep only + wgrad. Returns (gx, gparams)."""
        self._require()
        x = self._check_x(x)
        n = x.shape[0]
        gy = gy.contiguous()
        gx = torch.empty(n, self.cfg.d_in, dtype=torch.float32, device=x.device)
        gp = torch.empty(self.param_count, dtype=torch.float32, device=x.device)
        _lib.check(self.lib.siren_backward_stored(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(gy), _ptr(tws),
                                                  _ptr(gx), _ptr(gp), _stream(x.device)), 'siren_backward_stored')
        return gx, gp

    def second_order(self, ws, x, v, want_theta=True, gy=None, u=None, want_ydot=False, kept=None):
        """W3: the backward of the vjp node gx = J^T u (u (n, d_out), None = ones, i.e. diff_operators.gradient's
        dPhi/dx) given its cotangent v (n, d_in): H v and d/dtheta of F = sum <v, J^T u> (+ sum gy . y with a
        first-order seed gy (n, d_out)) in ONE sweep (siren_second_order_ex). Returns (gx, gparams or None), plus
        ydot = J v (n, d_out) = dF/du when want_ydot."""
        self._require()
        if not self.second_order_supported:
            raise _lib.SirenUnsupported('siren_second_order covers d_out <= 4, linear output, hidden 256 with 1..5 '
                                        'hidden layers (nonzero omegas beyond 3) or hidden 512')
        x = self._check_x(x)
        n, o = x.shape[0], self.cfg.d_out
        v = v.contiguous()
        if v.shape != x.shape or v.dtype != torch.float32 or v.device != x.device:
            raise ValueError('v must be fp32 %s on %s' % (tuple(x.shape), x.device))
        for name, t in (('gy', gy), ('u', u)):
            if t is not None and (t.numel() != n * o or t.dtype != torch.float32 or t.device != x.device):
                raise ValueError('%s must be fp32 with %d values on %s' % (name, n * o, x.device))
        gy = gy.contiguous() if gy is not None else None
        u = u.contiguous() if u is not None else None
        cnt = ctypes.c_int64()
        _lib.check(self.lib.siren_second_order_ws_floats(ctypes.byref(self.cfg), n, 1 if want_theta else 0,
                                                         ctypes.byref(cnt)), 'siren_second_order_ws_floats')
        tws = torch.empty(cnt.value, dtype=torch.float32, device=x.device)
        gx = torch.empty(n, self.cfg.d_in, dtype=torch.float32, device=x.device)
        gp = torch.empty(self.param_count, dtype=torch.float32, device=x.device) if want_theta else None
        ydot = torch.empty(n, o, dtype=torch.float32, device=x.device) if want_ydot else None
        if kept is not None and u is None and not want_ydot:
            # stored forward (forward_grad_store / forward_store): tangent-only hidden GEMMs
            _lib.check(self.lib.siren_second_order_kept(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(v), _ptr(gy),
                                                        _ptr(kept), _ptr(tws), _ptr(gx), _ptr(gp), _stream(x.device)),
                       'siren_second_order_kept')
            return gx, gp
        _lib.check(self.lib.siren_second_order_ex(ctypes.byref(self.cfg), _ptr(ws), _ptr(x), n, _ptr(v), _ptr(u),
                                                  _ptr(gy), _ptr(tws), _ptr(gx), _ptr(gp), _ptr(ydot),
                                                  _stream(x.device)), 'siren_second_order_ex')
        return (gx, gp, ydot) if want_ydot else (gx, gp)
