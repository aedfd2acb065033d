"""Drop-in SIREN modules: the reference's constructor signatures, parameter names and return values, with the
sine stack evaluated by the fused HIP kernels.

Mirrors (xvdp/siren):
  modules.py:11-25    BatchLinear          (nn.Linear + MetaModule; params= dict routing, batched weights)
  modules.py:28-34    Sine                 (sin(30 x))
  modules.py:37-116   FCBlock              (layer table, init, forward, forward_with_activations)
  modules.py:119-166  SingleBVPNet         (returns {'model_in', 'model_out'})
  modules.py:622-635  sine_init / first_layer_sine_init
  explore_siren.ipynb SineLayer / Siren    (configurable omega_0; forward returns (output, coords))
  torchmeta/modules/{module,container,utils}.py  MetaModule / MetaSequential / get_subdict
State-dict keys (net.net.{i}.0.weight|bias for SingleBVPNet, net.{i}.linear.* for Siren) and the RNG
consumption order of initialisation are the reference's, so torch.manual_seed(s) gives identical weights and
checkpoints load either way.

The fused path covers type='sine', mode='mlp', hidden_features 256 or 512, in/out_features <= 4, 1..8 hidden
layers (first-order derivatives at hidden 256: 1..3), unbatched fp32 weights on a ROCm device. A sine network outside that raises
SirenUnsupported; there is no silent torch or CPU fallback. Non-sine baselines (relu, tanh, ...) keep the
reference's plain torch layers: they are not the SIREN hot path.
"""
import math
import re
from collections import OrderedDict

import numpy as np
import torch
from torch import nn

from . import _lib
from .autograd import JetState, SirenBatchedFunction, SirenFunction, SirenJetFunction, SirenSplitFunction
from .engine import SirenEngine


# ----------------------------------------------------------------------------------------------------------
# torchmeta glue (torchmeta/modules/utils.py:4-11, module.py:6-27, container.py:6-19)
# ----------------------------------------------------------------------------------------------------------
def get_subdict(dictionary, key=None):
    """Sub-dictionary of `dictionary` whose keys start with `key.`, with that prefix stripped."""
    if dictionary is None:
        return None
    if key is None or key == '':
        return dictionary
    pat = re.compile(r'^' + re.escape(key) + r'\.(.+)')
    out = OrderedDict()
    for k, v in dictionary.items():
        m = pat.match(k)
        if m is not None:
            out[m.group(1)] = v
    return out


class MetaModule(nn.Module):
    """nn.Module whose forward accepts a `params` dict (meta-learning / hypernetwork protocol)."""

    def meta_named_parameters(self, prefix='', recurse=True):
        gen = self._named_members(lambda m: m._parameters.items() if isinstance(m, MetaModule) else [],
                                  prefix=prefix, recurse=recurse)
        yield from gen

    def meta_parameters(self, recurse=True):
        for _, p in self.meta_named_parameters(recurse=recurse):
            yield p


class MetaSequential(nn.Sequential, MetaModule):
    def forward(self, input, params=None):
        for name, module in self._modules.items():
            if isinstance(module, MetaModule):
                input = module(input, params=get_subdict(params, name))
            elif isinstance(module, nn.Module):
                input = module(input)
            else:
                raise TypeError('The module must be either a torch module (inheriting from `nn.Module`), or a '
                                '`MetaModule`. Got type: `{0}`'.format(type(module)))
        return input


# ----------------------------------------------------------------------------------------------------------
# layers
# ----------------------------------------------------------------------------------------------------------
class BatchLinear(nn.Linear, MetaModule):
    """nn.Linear that also takes (possibly batched, ...xOutxIn) weights through `params` (modules.py:11-25).
    Used on its own (and by non-sine baselines); inside a sine FCBlock the fused engine evaluates it."""
    __doc__ = nn.Linear.__doc__

    def forward(self, input, params=None):
        if params is None:
            params = OrderedDict(self.named_parameters())
        bias = params.get('bias', None)
        weight = params['weight']
        out = input.matmul(weight.transpose(-1, -2))
        if bias is not None:
            out = out + bias.unsqueeze(-2)
        return out


class Sine(nn.Module):
    """sin(30 x) (modules.py:28-34)."""

    def forward(self, input):
        return torch.sin(30 * input)


# ----------------------------------------------------------------------------------------------------------
# initialisation (modules.py:548-635)
# ----------------------------------------------------------------------------------------------------------
def _is_linear(m):
    return type(m) in (BatchLinear, nn.Linear)


def sine_init(m):
    with torch.no_grad():
        if hasattr(m, 'weight'):
            bound = np.sqrt(6 / m.weight.size(-1)) / 30
            m.weight.uniform_(-bound, bound)


def first_layer_sine_init(m):
    with torch.no_grad():
        if hasattr(m, 'weight'):
            fan_in = m.weight.size(-1)
            m.weight.uniform_(-1 / fan_in, 1 / fan_in)


def init_weights_normal(m):
    if _is_linear(m) and hasattr(m, 'weight'):
        nn.init.kaiming_normal_(m.weight, a=0.0, nonlinearity='relu', mode='fan_in')


def init_weights_selu(m):
    if _is_linear(m) and hasattr(m, 'weight'):
        nn.init.normal_(m.weight, std=1 / math.sqrt(m.weight.size(-1)))


def init_weights_elu(m):
    if _is_linear(m) and hasattr(m, 'weight'):
        nn.init.normal_(m.weight, std=math.sqrt(1.5505188080679277) / math.sqrt(m.weight.size(-1)))


def init_weights_xavier(m):
    if _is_linear(m) and hasattr(m, 'weight'):
        nn.init.xavier_normal_(m.weight)


# ----------------------------------------------------------------------------------------------------------
# engine cache + fused dispatch
# ----------------------------------------------------------------------------------------------------------
_ENGINES = {}


def get_engine(d_in, hidden, n_hidden, d_out, omega_first=30., omega_hidden=30., outermost_linear=True):
    key = (int(d_in), int(hidden), int(n_hidden), int(d_out), float(omega_first), float(omega_hidden),
           bool(outermost_linear))
    eng = _ENGINES.get(key)
    if eng is None:
        eng = _ENGINES[key] = SirenEngine(*key)
    return eng


PRECISIONS = ('fp32', 'bf16x6')


def _fused_apply(engine, jet, coords, weights_biases, precision='fp32'):
    """Run the fused SIREN on coords (..., d_in) with [(W, b), ...]; returns (..., d_out). precision 'bf16x6' runs
    the jet forward (y and dPhi/dx in one launch), a no-graph forward and a parameter-gradient training step
    (SirenSplitFunction) on the split-bf16 kernels where they cover the network; everything else
    stays on the fp32 kernels."""
    if coords.device.type != 'cuda':
        raise RuntimeError('siren_amd runs on ROCm devices (MI355X) only; move the model and coords to "cuda". '
                           'The CPU restatement of the reference lives in oracle/ (test infrastructure).')
    if not engine.supported:
        raise _lib.SirenUnsupported('siren_amd fused kernels do not cover this network: %s'
                                    % engine.unsupported_reason)
    if weights_biases[0][0].dim() == 3:
        return _fused_apply_batched(engine, coords, weights_biases)
    parts = []
    for W, b in weights_biases:
        if W.dim() != 2:
            raise _lib.SirenUnsupported('mixed batched / unbatched layer weights')
        parts.append(W.reshape(-1))
        parts.append(b.reshape(-1) if b is not None else W.new_zeros(W.shape[0]))
    flat = torch.cat(parts)
    lead = coords.shape[:-1]
    x2d = coords.reshape(-1, coords.shape[-1])
    if x2d is coords:  # keep a non-leaf edge so the engine can tell which gradients autograd wants
        x2d = coords.view(coords.shape)
    if (jet is not None and jet.active and engine.cfg.d_out == 1 and engine.grad_supported
            and torch.is_grad_enabled() and x2d.requires_grad):
        y, _ = SirenJetFunction.apply(engine, x2d, flat, flat.requires_grad,
                                      precision == 'bf16x6', jet)  # J: the node's second output
    elif (precision == 'bf16x6' and engine.split_supported
          and not (torch.is_grad_enabled() and (x2d.requires_grad or flat.requires_grad))):
        # no graph is recorded (dense evaluation: create_mesh, summaries under no_grad): the split-bf16 forward
        y = engine.forward_split(engine.pack_split(flat.detach()), x2d.detach().contiguous())
    elif (precision == 'bf16x6' and engine.split_supported and torch.is_grad_enabled() and flat.requires_grad
          and not (jet is not None and jet.laplace(JetState.key(x2d)))):
        # a training step: the split-bf16 forward and the bf16x6 W2 backward (a Laplacian consumer keeps the fp32
        # node, whose forward can speculate the jet sweep)
        y = SirenSplitFunction.apply(engine, jet, x2d, flat)
    else:
        # a graph that will want parameter gradients: the forward keeps a_l / cos for a reverse-only backward
        # (the jet state only matters when a graph is recorded: a derivative can be requested of y only then)
        y = SirenFunction.apply(engine, jet if torch.is_grad_enabled() else None, x2d, flat,
                                torch.is_grad_enabled() and flat.requires_grad)
    return y.view(*lead, y.shape[-1])


def _fused_apply_batched(engine, coords, weights_biases):
    """BatchLinear with batched weights (modules.py:16-25): W (B, out, in), b (B, out), coords (B, N, d_in) (or
    (1, N, d_in), broadcast over B as matmul does) -> (B, N, d_out) through SirenBatchedFunction."""
    B = weights_biases[0][0].shape[0]
    parts = []
    for W, b in weights_biases:
        if W.dim() != 3 or W.shape[0] != B:
            raise _lib.SirenUnsupported('batched weights need W (B, out, in) on every layer')
        parts.append(W.reshape(B, -1))
        parts.append(b.reshape(B, -1) if b is not None else W.new_zeros(B, W.shape[1]))
    flat = torch.cat(parts, dim=1)
    if coords.dim() != 3:
        raise _lib.SirenUnsupported('batched weights need coords of shape (B, N, d_in)')
    x = coords.expand(B, -1, -1) if coords.shape[0] == 1 and B > 1 else coords
    if x.shape[0] != B:
        raise ValueError('coords batch %d does not match the weights batch %d' % (x.shape[0], B))
    if x is coords:
        x = coords.view(coords.shape)  # a non-leaf edge, as in _fused_apply
    return SirenBatchedFunction.apply(engine, x, flat, torch.is_grad_enabled() and flat.requires_grad)


# ----------------------------------------------------------------------------------------------------------
# FCBlock / SingleBVPNet (modules.py:37-166)
# ----------------------------------------------------------------------------------------------------------
class FCBlock(MetaModule):
    """Fully connected block; with nonlinearity='sine' it is evaluated by the fused engine."""

    def __init__(self, in_features, out_features, num_hidden_layers, hidden_features, outermost_linear=False,
                 nonlinearity='relu', weight_init=None, jet='auto', precision='fp32'):
        super().__init__()
        if precision not in PRECISIONS:
            raise ValueError('precision must be one of %s; got %r' % (PRECISIONS, precision))
        self.precision = precision
        self.first_layer_init = None
        table = {'sine': (Sine(), sine_init, first_layer_sine_init),
                 'relu': (nn.ReLU(inplace=True), init_weights_normal, None),
                 'sigmoid': (nn.Sigmoid(), init_weights_xavier, None),
                 'tanh': (nn.Tanh(), init_weights_xavier, None),
                 'selu': (nn.SELU(inplace=True), init_weights_selu, None),
                 'softplus': (nn.Softplus(), init_weights_normal, None),
                 'elu': (nn.ELU(inplace=True), init_weights_elu, None)}
        nl, nl_weight_init, first_layer_init = table[nonlinearity]
        self.nonlinearity = nonlinearity
        self.weight_init = weight_init if weight_init is not None else nl_weight_init
        self.in_features, self.out_features = in_features, out_features
        self.hidden_features, self.num_hidden_layers = hidden_features, num_hidden_layers
        self.outermost_linear = outermost_linear

        layers = [MetaSequential(BatchLinear(in_features, hidden_features), nl)]
        for _ in range(num_hidden_layers):
            layers.append(MetaSequential(BatchLinear(hidden_features, hidden_features), nl))
        if outermost_linear:
            layers.append(MetaSequential(BatchLinear(hidden_features, out_features)))
        else:
            layers.append(MetaSequential(BatchLinear(hidden_features, out_features), nl))
        self.net = MetaSequential(*layers)
        if self.weight_init is not None:
            self.net.apply(self.weight_init)
        if first_layer_init is not None:
            self.net[0].apply(first_layer_init)
        self._jet = JetState(jet)

    def _engine(self):
        return get_engine(self.in_features, self.hidden_features, self.num_hidden_layers, self.out_features,
                          30., 30., self.outermost_linear)

    def forward(self, coords, params=None, **kwargs):
        if params is None:
            params = OrderedDict(self.named_parameters())
        params = get_subdict(params, 'net')
        if self.nonlinearity != 'sine':
            return self.net(coords, params=params)
        wb = [(params['%d.0.weight' % i], params.get('%d.0.bias' % i)) for i in range(len(self.net))]
        return _fused_apply(self._engine(), self._jet, coords, wb, self.precision)

    def forward_with_activations(self, coords, params=None, retain_grad=False):
        """Per-layer activations (modules.py:96-116): a visualisation API, evaluated layer by layer in torch."""
        if params is None:
            params = OrderedDict(self.named_parameters())
        activations = OrderedDict()
        x = coords.clone().detach().requires_grad_(True)
        activations['input'] = x
        for i, layer in enumerate(self.net):
            sub = get_subdict(params, 'net.%d' % i)
            for j, sublayer in enumerate(layer):
                if isinstance(sublayer, BatchLinear):
                    x = sublayer(x, params=get_subdict(sub, '%d' % j))
                else:
                    x = sublayer(x)
                if retain_grad:
                    x.retain_grad()
                activations['_'.join((str(sublayer.__class__), '%d' % i))] = x
        return activations


class SingleBVPNet(MetaModule):
    """A canonical representation network for a BVP (modules.py:119-166).

    forward(model_input: {'coords': (B, N, d)}, params=None) -> {'model_in': (B, N, d) leaf with
    requires_grad, 'model_out': (B, N, out_features)}; 'coords' is an alias of 'model_in'.
    Extra keyword `jet` ('auto' | True | False): compute dPhi/dx in the forward launch (W1 kernel) so that
    diff_operators.gradient costs no second sweep; 'auto' switches it on after the first such request.
    Extra keyword `precision` ('fp32' | 'bf16x6'): 'bf16x6' evaluates that jet forward on the split-bf16 kernel
    (fp32 operands split exactly into bf16 hi/mid/lo, fp32-level error, 1.6x the fp32 kernel at 5x256 d2/d3 o1)
    where it covers the network, and a forward that records no graph (no_grad: create_mesh, summaries) on the split
    W0 kernel (1.85x), and a step whose loss needs parameter gradients of model_out only (image fitting) on the
    split W0 forward plus the bf16x6 W2 backward (siren_backward_split: split-bf16 recompute + reverse, fp32 MFMA
    wgrad). A backward through the jet node recomputes on the fp32 kernels.
    """

    def __init__(self, out_features=1, type='sine', in_features=2, mode='mlp', hidden_features=256,
                 num_hidden_layers=3, **kwargs):
        super().__init__()
        self.mode = mode
        if mode != 'mlp':
            raise _lib.SirenUnsupported("siren_amd covers mode='mlp' (rbf/nerf input encodings are out of scope)")
        if kwargs.get('downsample', False):
            raise _lib.SirenUnsupported('ImageDownsampling jitter (downsample=True) is out of scope')
        self.net = FCBlock(in_features=in_features, out_features=out_features, num_hidden_layers=num_hidden_layers,
                           hidden_features=hidden_features, outermost_linear=True, nonlinearity=type,
                           jet=kwargs.get('jet', 'auto'), precision=kwargs.get('precision', 'fp32'))
        if kwargs.get('verbose', True):
            print(self)

    def forward(self, model_input, params=None):
        if params is None:
            params = OrderedDict(self.named_parameters())
        coords_org = model_input['coords'].clone().detach().requires_grad_(True)
        output = self.net(coords_org, get_subdict(params, 'net'))
        return {'model_in': coords_org, 'model_out': output, 'coords': coords_org}

    def forward_with_activations(self, model_input):
        coords = model_input['coords'].clone().detach().requires_grad_(True)
        activations = self.net.forward_with_activations(coords)
        return {'model_in': coords, 'model_out': activations.popitem(), 'activations': activations}


# ----------------------------------------------------------------------------------------------------------
# notebook API: SineLayer / Siren (explore_siren.ipynb)
# ----------------------------------------------------------------------------------------------------------
class SineLayer(nn.Module):
    """sin(omega_0 (x W^T + b)); first layer init U(+-1/in), others U(+-sqrt(6/in)/omega_0)."""

    def __init__(self, in_features, out_features, bias=True, is_first=False, omega_0=30):
        super().__init__()
        self.omega_0 = omega_0
        self.is_first = is_first
        self.in_features = in_features
        self.linear = nn.Linear(in_features, out_features, bias=bias)
        self.init_weights()

    def init_weights(self):
        with torch.no_grad():
            if self.is_first:
                self.linear.weight.uniform_(-1 / self.in_features, 1 / self.in_features)
            else:
                b = np.sqrt(6 / self.in_features) / self.omega_0
                self.linear.weight.uniform_(-b, b)

    def forward(self, input):
        return torch.sin(self.omega_0 * self.linear(input))

    def forward_with_intermediate(self, input):
        intermediate = self.omega_0 * self.linear(input)
        return torch.sin(intermediate), intermediate


class Siren(nn.Module):
    """Notebook Siren: forward(coords) -> (output, coords) with coords a fresh leaf requiring grad."""

    def __init__(self, in_features, hidden_features, hidden_layers, out_features, outermost_linear=False,
                 first_omega_0=30, hidden_omega_0=30., jet='auto'):
        super().__init__()
        self.in_features, self.hidden_features, self.hidden_layers = in_features, hidden_features, hidden_layers
        self.out_features, self.outermost_linear = out_features, outermost_linear
        self.first_omega_0, self.hidden_omega_0 = first_omega_0, hidden_omega_0
        net = [SineLayer(in_features, hidden_features, is_first=True, omega_0=first_omega_0)]
        for _ in range(hidden_layers):
            net.append(SineLayer(hidden_features, hidden_features, is_first=False, omega_0=hidden_omega_0))
        if outermost_linear:
            final_linear = nn.Linear(hidden_features, out_features)
            with torch.no_grad():
                b = np.sqrt(6 / hidden_features) / hidden_omega_0
                final_linear.weight.uniform_(-b, b)
            net.append(final_linear)
        else:
            net.append(SineLayer(hidden_features, out_features, is_first=False, omega_0=hidden_omega_0))
        self.net = nn.Sequential(*net)
        self._jet = JetState(jet)

    def _weights(self):
        out = []
        for layer in self.net:
            lin = layer.linear if isinstance(layer, SineLayer) else layer
            out.append((lin.weight, lin.bias))
        return out

    def forward(self, coords):
        coords = coords.clone().detach().requires_grad_(True)
        eng = get_engine(self.in_features, self.hidden_features, self.hidden_layers, self.out_features,
                         self.first_omega_0, self.hidden_omega_0, self.outermost_linear)
        return _fused_apply(eng, self._jet, coords, self._weights()), coords

    def forward_with_activations(self, coords, retain_grad=False):
        activations = OrderedDict()
        count = 0
        x = coords.clone().detach().requires_grad_(True)
        activations['input'] = x
        for layer in self.net:
            if isinstance(layer, SineLayer):
                x, intermed = layer.forward_with_intermediate(x)
                if retain_grad:
                    x.retain_grad()
                    intermed.retain_grad()
                activations['_'.join((str(layer.__class__), '%d' % count))] = intermed
                count += 1
            else:
                x = layer(x)
                if retain_grad:
                    x.retain_grad()
            activations['_'.join((str(layer.__class__), '%d' % count))] = x
            count += 1
        return activations


# ----------------------------------------------------------------------------------------------------------
# Complex helpers of the PML losses (modules.py:636-673): a complex field is stored as interleaved channels
# (re_0, im_0, re_1, im_1, ...) along the last dimension.
# ----------------------------------------------------------------------------------------------------------
def _interleave(re, im):
    return torch.stack((re, im), dim=-1).flatten(-2)


def compl_conj(x):
    """Complex conjugate: negate the odd (imaginary) channels."""
    return _interleave(x[..., ::2], -x[..., 1::2])


def compl_div(x, y):
    """x / y channel-pair-wise: ((ac + bd) + i (bc - ad)) / (c^2 + d^2)."""
    a, b, c, d = x[..., ::2], x[..., 1::2], y[..., ::2], y[..., 1::2]
    den = c ** 2 + d ** 2
    return _interleave((a * c + b * d) / den, (b * c - a * d) / den)


def compl_mul(x, y):
    """x * y channel-pair-wise; the imaginary part uses the reference's three-multiplication form
    (a + b)(c + d) - ac - bd, so the rounding matches."""
    a, b, c, d = x[..., ::2], x[..., 1::2], y[..., ::2], y[..., 1::2]
    ac, bd = a * c, b * d
    return _interleave(ac - bd, (a + b) * (c + d) - ac - bd)
