"""HyperNetwork (meta_modules.py:10-53, 136-154): one ReLU FCBlock per parameter of a hypo-network predicts that
parameter, batched over the embedding rows. Its output dict goes straight to SingleBVPNet/FCBlock(params=...),
where the batched-weights path (SirenBatchedFunction: one grouped W0 / W1 launch over the batch, W2 per element)
evaluates the SIREN. The hypernetwork itself is a small ReLU MLP kept as plain torch layers (not the hot path)."""
from collections import OrderedDict

import torch
from torch import nn

from . import modules


def hyper_weight_init(m, in_features_main_net):
    """Kaiming-normal / 100 weights, biases U(+-1/in_features of the hypo layer) (meta_modules.py:136-143)."""
    if hasattr(m, 'weight'):
        nn.init.kaiming_normal_(m.weight, a=0.0, nonlinearity='relu', mode='fan_in')
        m.weight.data = m.weight.data / 1.e2
    if hasattr(m, 'bias'):
        with torch.no_grad():
            m.bias.uniform_(-1 / in_features_main_net, 1 / in_features_main_net)


def hyper_bias_init(m):
    """Kaiming-normal / 100 weights, biases U(+-1/fan_in) (meta_modules.py:146-154)."""
    if hasattr(m, 'weight'):
        nn.init.kaiming_normal_(m.weight, a=0.0, nonlinearity='relu', mode='fan_in')
        m.weight.data = m.weight.data / 1.e2
    if hasattr(m, 'bias'):
        fan_in, _ = nn.init._calculate_fan_in_and_fan_out(m.weight)
        with torch.no_grad():
            m.bias.uniform_(-1 / fan_in, 1 / fan_in)


class HyperNetwork(nn.Module):
    """HyperNetwork(hyper_in_features, hyper_hidden_layers, hyper_hidden_features, hypo_module): forward(z (B, in))
    -> OrderedDict name -> (B, *param_shape), in hypo_module.meta_named_parameters() order."""

    def __init__(self, hyper_in_features, hyper_hidden_layers, hyper_hidden_features, hypo_module):
        super().__init__()
        self.names, self.param_shapes = [], []
        self.nets = nn.ModuleList()
        for name, param in hypo_module.meta_named_parameters():
            self.names.append(name)
            self.param_shapes.append(param.size())
            hn = modules.FCBlock(in_features=hyper_in_features, out_features=int(param.numel()),
                                 num_hidden_layers=hyper_hidden_layers, hidden_features=hyper_hidden_features,
                                 outermost_linear=True, nonlinearity='relu')
            self.nets.append(hn)
            last = self.nets[-1].net[-1]
            if 'weight' in name:
                last.apply(lambda m, fi=param.size()[-1]: hyper_weight_init(m, fi))
            elif 'bias' in name:
                last.apply(hyper_bias_init)

    def forward(self, z):
        params = OrderedDict()
        for name, net, shape in zip(self.names, self.nets, self.param_shapes):
            params[name] = net(z).reshape((-1,) + tuple(shape))
        return params
