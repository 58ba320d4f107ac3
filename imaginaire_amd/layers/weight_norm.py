"""Weight normalisations (reference layers/weight_norm.py:14-92).

``spectral`` uses PyTorch's spectral-norm parametrisation so checkpoints keep
the reference's ``weight_orig / weight_u / weight_v`` keys; ``get_weight``
exposes the normalised weight so fused paths (e.g. the γ|β conv of SPADE) can
concatenate several normalised weights into one MIOpen call.
"""
import functools

import torch
from torch import nn
from torch.nn.utils import weight_norm
from torch.nn.utils.spectral_norm import SpectralNorm as _TorchSN

from .conv import LinearBlock
from .spectral_norm import spectral_norm


from torch.nn.utils.weight_norm import WeightNorm as _TorchWN


def _sn_hook(module):
    for hook in module._forward_pre_hooks.values():
        if isinstance(hook, _TorchSN):
            return hook
    return None


def _wn_hook(module):
    for hook in module._forward_pre_hooks.values():
        if isinstance(hook, _TorchWN):
            return hook
    return None


def get_weight(module, ref=False):
    """Effective weight of a conv/linear, running one SN power iteration in training.

    Mirrors what the module's own forward would use; call at most once per
    forward pass per module (the power iteration updates ``weight_u``).
    ``ref=True`` (callers that hand the weight straight to ``ops.conv.conv2d`` /
    ``conv2d_act``): a spectrally normalised plain Conv2d whose batched iteration left its
    W / sigma unmaterialised comes back as an ``ops.conv.SNWeight`` — the conv then runs on the
    bf16 shadow with 1 / sigma in its epilogue and the SN backward folded into its weight
    gradient (layers/spectral_norm.py).
    """
    hook = _sn_hook(module)
    if hook is not None:
        if ref and hasattr(hook, 'weight_ref'):
            r = hook.weight_ref(module)
            if r is not None:
                # module.weight must not keep a stale tensor (torch's spectral_norm leaves the
                # forward's W / sigma there): it holds the unmaterialised reference, whose
                # .materialize() gives bf16(W / sigma)
                setattr(module, hook.name, r)
                return r
        w = hook.compute_weight(module, do_power_iteration=module.training)
        setattr(module, hook.name, w)
        return w
    hook = _wn_hook(module)
    if hook is not None:
        w = hook.compute_weight(module)
        setattr(module, hook.name, w)
        return w
    return module.weight


def has_spectral_norm(module):
    return _sn_hook(module) is not None


class WeightDemodulation(nn.Module):
    """StyleGAN2 modulated / demodulated convolution (weight_norm.py:14-63). On the GPU the
    per-sample modulated weights feed the batched per-sample k10 convolution (the hyper-conv
    path of few-shot vid2vid, ``ops/conv.py: conv2d_per_sample``)."""

    def __init__(self, conv, cond_dims, eps=1e-8, adaptive_bias=False, demod=True):
        super().__init__()
        self.conv = conv
        self.adaptive_bias = adaptive_bias
        if adaptive_bias:
            self.conv.register_parameter('bias', None)
            self.fc_beta = LinearBlock(cond_dims, self.conv.out_channels)
        self.fc_gamma = LinearBlock(cond_dims, self.conv.in_channels)
        self.eps = eps
        self.demod = demod
        self.conditional = True

    def forward(self, x, y):
        b, c, h, w = x.size()
        gamma = self.fc_gamma(y)[:, None, :, None, None]
        weight = self.conv.weight[None] * (gamma + 1)
        if self.demod:
            d = torch.rsqrt((weight ** 2).sum(dim=(2, 3, 4), keepdim=True) + self.eps)
            weight = weight * d
        from imaginaire_amd.ops import conv as conv_ops
        stride = self.conv.stride[0] if self.conv.stride[0] == self.conv.stride[1] else None
        if isinstance(self.conv.padding, tuple) and stride == 1 and \
                conv_ops.per_sample_eligible(x, weight, stride, 1):
            # per-sample (modulated) weights as ONE batched k10 launch, grid z = sample (and
            # batched k10 / k11 backward), instead of a b-group MIOpen convolution
            bias = self.conv.bias[None].expand(b, -1) if self.conv.bias is not None else None
            x = conv_ops.conv2d_per_sample(x, weight, bias, self.conv.padding,
                                           self.conv.dilation)
        else:
            x = x.reshape(1, -1, h, w)
            _, _, *ws = weight.shape
            weight = weight.reshape(b * self.conv.out_channels, *ws)
            bias = self.conv.bias.repeat(b) if self.conv.bias is not None else None
            x = conv_ops.conv2d(x, weight, bias, self.conv.stride, self.conv.padding,
                                self.conv.dilation, groups=b)
            x = x.reshape(-1, self.conv.out_channels, x.shape[2], x.shape[3])
        if self.adaptive_bias:
            x = x + self.fc_beta(y)[:, :, None, None]
        return x


def weight_demod(conv, cond_dims=256, eps=1e-8, demod=True):
    return WeightDemodulation(conv, cond_dims, eps, demod=demod)


def get_weight_norm_layer(norm_type, **norm_params):
    """Return a function that wraps a conv/linear with weight normalisation."""
    if norm_type == 'none' or norm_type == '':
        return lambda x: x
    if norm_type == 'spectral':
        return functools.partial(spectral_norm, **norm_params)
    if norm_type == 'weight':
        return functools.partial(weight_norm, **norm_params)
    if norm_type == 'weight_demod':
        return functools.partial(weight_demod, **norm_params)
    raise ValueError('Weight norm layer %s is not recognized' % norm_type)
