"""Nonlinearity factory (reference layers/nonlinearity.py:8-37).

``act_slope`` maps a nonlinearity module to the leaky slope the fused HIP
kernels understand (relu → 0, leakyrelu → its negative slope, none → 1), or
``None`` if it cannot be fused (prelu / tanh / sigmoid / softmax).
"""
from torch import nn


def get_nonlinearity_layer(nonlinearity_type, inplace):
    if nonlinearity_type == 'relu':
        return nn.ReLU(inplace=inplace)
    if nonlinearity_type == 'leakyrelu':
        return nn.LeakyReLU(0.2, inplace=inplace)
    if nonlinearity_type == 'prelu':
        return nn.PReLU()
    if nonlinearity_type == 'tanh':
        return nn.Tanh()
    if nonlinearity_type == 'sigmoid':
        return nn.Sigmoid()
    if nonlinearity_type.startswith('softmax'):
        dim = nonlinearity_type.split(',')[1] if ',' in nonlinearity_type else 1
        return nn.Softmax(dim=int(dim))
    if nonlinearity_type == 'none' or nonlinearity_type == '':
        return None
    raise ValueError('Nonlinearity %s is not recognized' % nonlinearity_type)


def act_slope(layer):
    if layer is None:
        return 1.0
    if isinstance(layer, nn.LeakyReLU):
        return float(layer.negative_slope)
    if isinstance(layer, nn.ReLU):
        return 0.0
    return None
