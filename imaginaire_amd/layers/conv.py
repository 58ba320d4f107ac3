"""Convolution blocks (reference layers/conv.py:14-1072).

A block is ``{conv [+noise], norm, activation}`` applied in the order given by
an ``order`` string (``'CNA'``, ``'NAC'``, ``'ANC'``, ...), with the reference's
module names (``layers.conv`` / ``layers.norm`` / ``layers.nonlinearity``) so
checkpoints are interchangeable.

MI355X execution plan (decided per forward from the module types):
  * ``N`` immediately followed by a leaky/relu ``A`` → one fused HIP
    norm(+SPADE/AdaIN modulation)+activation kernel (k1, ops/norm.py);
  * ``C`` immediately followed by a leaky/relu ``A`` (no norm between) → one
    MFMA implicit-GEMM conv with the bias+activation in its epilogue (k10,
    ops/conv.py) when eligible, else bias-free MIOpen conv + fused bias+activation
    HIP epilogue (k2, ops/bias_act.py);
  * everything else runs the module as is.
"""
from types import SimpleNamespace

import torch
from torch import nn
from torch.nn import functional as F

from imaginaire_amd.ops import conv as nhwc_conv
from imaginaire_amd.ops.bias_act import bias_act
from imaginaire_amd.ops.partial_conv import partial_conv_renorm
from .misc import ApplyNoise
from .nonlinearity import act_slope


def _plain_conv_weight(conv):
    from .weight_norm import get_weight
    # (an ops.conv.SNWeight for a batched spectral-norm conv: the conv ops take it as is)
    return get_weight(conv, ref=isinstance(conv, nn.Conv2d))


def _fusible_conv(layer):
    return isinstance(layer, (nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.Linear)) and \
        type(layer) in (nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.Linear) and \
        getattr(layer, 'padding_mode', 'zeros') == 'zeros' and \
        getattr(layer, 'bias', None) is not None and \
        not any(isinstance(h, nn.Module) for h in layer._forward_hooks.values())


def _conv_nobias(layer, x):
    w = _plain_conv_weight(layer)
    if isinstance(w, nhwc_conv.SNWeight) and not isinstance(layer, nn.Conv2d):
        w = w.materialize()
    if isinstance(layer, nn.Linear):
        return F.linear(x, w, None)
    if isinstance(layer, nn.Conv2d):
        return nhwc_conv.conv2d(x, w, None, layer.stride, layer.padding, layer.dilation,
                                layer.groups)
    if isinstance(layer, nn.Conv1d):
        return F.conv1d(x, w, None, layer.stride, layer.padding, layer.dilation, layer.groups)
    return F.conv3d(x, w, None, layer.stride, layer.padding, layer.dilation, layer.groups)


def _is_plain_conv2d(layer):
    return type(layer) is nn.Conv2d and \
        not any(isinstance(h, nn.Module) for h in layer._forward_hooks.values())


class _BaseConvBlock(nn.Module):
    """Conv/linear + noise + norm + nonlinearity in a configurable order."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, dilation,
                 groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                 activation_norm_type, activation_norm_params, nonlinearity,
                 inplace_nonlinearity, apply_noise, order, input_dim):
        super().__init__()
        from .nonlinearity import get_nonlinearity_layer
        from .weight_norm import get_weight_norm_layer
        from .activation_norm import get_activation_norm_layer
        self.weight_norm_type = weight_norm_type
        if weight_norm_params is None:
            weight_norm_params = SimpleNamespace()
        weight_norm = get_weight_norm_layer(weight_norm_type, **vars(weight_norm_params))
        conv_layer = weight_norm(self._get_conv_layer(
            in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias,
            padding_mode, input_dim))
        noise_layer = ApplyNoise() if apply_noise else None
        conv_before_norm = order.find('C') < order.find('N')
        norm_channels = out_channels if conv_before_norm else in_channels
        if activation_norm_params is None:
            activation_norm_params = SimpleNamespace()
        activation_norm_layer = get_activation_norm_layer(
            norm_channels, activation_norm_type, input_dim, **vars(activation_norm_params))
        nonlinearity_layer = get_nonlinearity_layer(nonlinearity, inplace=inplace_nonlinearity)
        mappings = {'C': {'conv': conv_layer},
                    'N': {'norm': activation_norm_layer},
                    'A': {'nonlinearity': nonlinearity_layer}}
        self.layers = nn.ModuleDict()
        for op in order:
            if list(mappings[op].values())[0] is not None:
                self.layers.update(mappings[op])
                if op == 'C' and noise_layer is not None:
                    self.layers.update({'noise': noise_layer})
        self.conditional = getattr(conv_layer, 'conditional', False) or \
            getattr(activation_norm_layer, 'conditional', False)

    def forward(self, x, *cond_inputs, residual=None, skip_first_act=False, **kw_cond_inputs):
        """``residual``: added to the block's output (a residual block's shortcut). When the
        block ends in a plain 2-D conv it lands in the k10 epilogue (ops/conv.py ``conv2d``).
        ``skip_first_act``: the caller already applied the block's leading nonlinearity (an
        'A..' order block; e.g. before a nearest upsampling it commutes with, on 4x fewer
        pixels)."""
        keys = list(self.layers.keys())
        i = 1 if (skip_first_act and keys and keys[0] == 'nonlinearity') else 0
        n = len(keys)
        while i < n:
            name = keys[i]
            layer = self.layers[name]
            nxt = keys[i + 1] if i + 1 < n else None
            if nxt == 'nonlinearity':
                slope = act_slope(self.layers['nonlinearity'])
                if slope is not None:
                    if name == 'norm' and getattr(layer, 'supports_fused_act', False):
                        if getattr(layer, 'conditional', False):
                            x = layer(x, *cond_inputs, act_slope=slope, **kw_cond_inputs)
                        else:
                            x = layer(x, act_slope=slope)
                        i += 2
                        continue
                    if name == 'conv' and _fusible_conv(layer):
                        if isinstance(layer, nn.Conv2d) and x.is_cuda:
                            x = nhwc_conv.conv2d_act(x, _plain_conv_weight(layer), layer.bias,
                                                     layer.stride, layer.padding, layer.dilation,
                                                     slope) if layer.groups == 1 else \
                                bias_act(_conv_nobias(layer, x), layer.bias, slope)
                        else:
                            x = bias_act(_conv_nobias(layer, x), layer.bias, slope)
                        i += 2
                        continue
            if name == 'conv' and _is_plain_conv2d(layer) and x.is_cuda:
                last = i + 1 == n
                x = nhwc_conv.conv2d(x, _plain_conv_weight(layer), layer.bias, layer.stride,
                                     layer.padding, layer.dilation, layer.groups,
                                     layer.padding_mode, residual=residual if last else None)
                if last:
                    residual = None
            elif getattr(layer, 'conditional', False):
                x = layer(x, *cond_inputs, **kw_cond_inputs)
            else:
                x = layer(x)
            i += 1
        if residual is not None:
            x = x + residual
        return x

    def _get_conv_layer(self, in_channels, out_channels, kernel_size, stride, padding,
                        dilation, groups, bias, padding_mode, input_dim):
        if input_dim == 0:
            return nn.Linear(in_channels, out_channels, bias)
        layer_type = getattr(nn, 'Conv%dd' % input_dim)
        return layer_type(in_channels, out_channels, kernel_size, stride, padding, dilation,
                          groups, bias, padding_mode)

    def __repr__(self):
        main_str = self._get_name() + '('
        child_lines = []
        for name, layer in self.layers.items():
            mod_str = repr(layer)
            if name == 'conv' and self.weight_norm_type not in ('none', ''):
                mod_str = mod_str[:-1] + ', weight_norm={}'.format(self.weight_norm_type) + ')'
            child_lines.append(_addindent(mod_str, 2))
        if len(child_lines) == 1:
            main_str += child_lines[0]
        else:
            main_str += '\n  ' + '\n  '.join(child_lines) + '\n'
        return main_str + ')'


def _addindent(s_, num_spaces):
    s = s_.split('\n')
    if len(s) == 1:
        return s_
    first = s.pop(0)
    return first + '\n' + '\n'.join((num_spaces * ' ') + line for line in s)


class LinearBlock(_BaseConvBlock):
    def __init__(self, in_features, out_features, bias=True, weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, nonlinearity='none', inplace_nonlinearity=False,
                 apply_noise=False, order='CNA'):
        super().__init__(in_features, out_features, None, None, None, None, None, bias, None,
                         weight_norm_type, weight_norm_params, activation_norm_type,
                         activation_norm_params, nonlinearity, inplace_nonlinearity,
                         apply_noise, order, 0)


class Conv1dBlock(_BaseConvBlock):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, padding_mode='zeros', weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, nonlinearity='none', inplace_nonlinearity=False,
                 apply_noise=False, order='CNA'):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation,
                         groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, nonlinearity,
                         inplace_nonlinearity, apply_noise, order, 1)


class Conv2dBlock(_BaseConvBlock):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, padding_mode='zeros', weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, nonlinearity='none', inplace_nonlinearity=False,
                 apply_noise=False, order='CNA'):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation,
                         groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, nonlinearity,
                         inplace_nonlinearity, apply_noise, order, 2)


class Conv3dBlock(_BaseConvBlock):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, padding_mode='zeros', weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, nonlinearity='none', inplace_nonlinearity=False,
                 apply_noise=False, order='CNA'):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation,
                         groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, nonlinearity,
                         inplace_nonlinearity, apply_noise, order, 3)


class _BaseHyperConvBlock(_BaseConvBlock):
    """Block whose conv and/or norm weights are supplied at run time (conv.py:399-447)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, dilation,
                 groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                 activation_norm_type, activation_norm_params, nonlinearity,
                 inplace_nonlinearity, apply_noise, is_hyper_conv, is_hyper_norm, order,
                 input_dim):
        self.is_hyper_conv = is_hyper_conv
        if is_hyper_conv:
            weight_norm_type = 'none'
        if is_hyper_norm:
            activation_norm_type = 'hyper_' + activation_norm_type
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation,
                         groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, nonlinearity,
                         inplace_nonlinearity, apply_noise, order, input_dim)

    def _get_conv_layer(self, in_channels, out_channels, kernel_size, stride, padding,
                        dilation, groups, bias, padding_mode, input_dim):
        if input_dim == 0:
            raise ValueError('HyperLinearBlock is not supported.')
        if self.is_hyper_conv:
            return HyperConv2d(in_channels, out_channels, kernel_size, stride, padding, dilation,
                               groups, bias, padding_mode)
        return getattr(nn, 'Conv%dd' % input_dim)(in_channels, out_channels, kernel_size, stride,
                                                  padding, dilation, groups, bias, padding_mode)


class HyperConv2dBlock(_BaseHyperConvBlock):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, padding_mode='zeros', weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, is_hyper_conv=False, is_hyper_norm=False,
                 nonlinearity='none', inplace_nonlinearity=False, apply_noise=False,
                 order='CNA'):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation,
                         groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, nonlinearity,
                         inplace_nonlinearity, apply_noise, is_hyper_conv, is_hyper_norm,
                         order, 2)


class HyperConv2d(nn.Module):
    """Convolution with per-sample weights supplied at run time (conv.py:511-590).

    The reference loops over the batch issuing one conv per sample; here the
    batch is folded into the channel axis and one grouped MIOpen convolution
    (groups = B·groups) runs all samples at once.
    """

    def __init__(self, in_channels=0, out_channels=0, kernel_size=3, stride=1, padding=1,
                 dilation=1, groups=1, bias=True, padding_mode='zeros'):
        super().__init__()
        self.stride = stride
        self.padding = padding
        self.dilation = dilation
        self.groups = groups
        self.use_bias = bias
        self.padding_mode = padding_mode
        self.conditional = True

    def forward(self, x, *args, conv_weights=(None, None), **kwargs):
        if conv_weights is None:
            conv_weight, conv_bias = None, None
        elif isinstance(conv_weights, torch.Tensor):
            conv_weight, conv_bias = conv_weights, None
        else:
            conv_weight, conv_bias = conv_weights
        if conv_weight is None:
            return x
        b = x.size(0)
        if conv_bias is None and self.use_bias:
            raise ValueError('bias not provided but set to true during initialization')
        if self.padding_mode != 'zeros':
            x = nhwc_conv.pad(nhwc_conv.nhwc(x), [self.padding] * 4, self.padding_mode)
            padding = 0
        else:
            padding = self.padding
        if conv_weight.dim() == 4:
            conv_weight = conv_weight.unsqueeze(0).expand(b, *conv_weight.shape)
        if self.stride == 1 and nhwc_conv.per_sample_eligible(x, conv_weight, self.stride,
                                                               self.groups):
            # one batched k10 launch (grid z = sample) instead of a grouped MIOpen conv
            bias = conv_bias.reshape(b, -1) if conv_bias is not None else None
            return nhwc_conv.conv2d_per_sample(nhwc_conv.nhwc(x), conv_weight, bias, padding,
                                               self.dilation)
        xg = x.reshape(1, b * x.size(1), x.size(2), x.size(3))
        if self.stride >= 1:
            w = conv_weight.reshape(b * conv_weight.size(1), *conv_weight.shape[2:])
            bias = conv_bias.reshape(-1) if conv_bias is not None else None
            y = nhwc_conv.conv2d(xg, w, bias, stride=self.stride, padding=padding,
                                 dilation=self.dilation, groups=b * self.groups)
        else:
            w = conv_weight.reshape(b * conv_weight.size(1), *conv_weight.shape[2:])
            bias = conv_bias.reshape(-1) if conv_bias is not None else None
            y = nhwc_conv.conv_transpose2d(xg, w, bias, stride=int(1 / self.stride),
                                           padding=self.padding, output_padding=self.padding,
                                           groups=b * self.groups, dilation=self.dilation)
        return y.reshape(b, -1, y.size(2), y.size(3))


class _BasePartialConvBlock(_BaseConvBlock):
    """Partial-convolution block (conv.py:593-657)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, dilation,
                 groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                 activation_norm_type, activation_norm_params, nonlinearity,
                 inplace_nonlinearity, multi_channel, return_mask, apply_noise, order,
                 input_dim):
        self.multi_channel = multi_channel
        self.return_mask = return_mask
        self.partial_conv = True
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation,
                         groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, nonlinearity,
                         inplace_nonlinearity, apply_noise, order, input_dim)

    def _get_conv_layer(self, in_channels, out_channels, kernel_size, stride, padding,
                        dilation, groups, bias, padding_mode, input_dim):
        if input_dim == 2:
            layer_type = PartialConv2d
        elif input_dim == 3:
            layer_type = PartialConv3d
        else:
            raise ValueError('Partial conv only supports 2D and 3D conv now.')
        return layer_type(in_channels, out_channels, kernel_size, stride, padding, dilation,
                          groups, bias, padding_mode, multi_channel=self.multi_channel,
                          return_mask=self.return_mask)

    def forward(self, x, *cond_inputs, mask_in=None, **kw_cond_inputs):
        mask_out = None
        for layer in self.layers.values():
            if getattr(layer, 'conditional', False):
                x = layer(x, *cond_inputs, **kw_cond_inputs)
            elif getattr(layer, 'partial_conv', False):
                x = layer(x, mask_in=mask_in, **kw_cond_inputs)
                if type(x) == tuple:
                    x, mask_out = x
            else:
                x = layer(x)
        if mask_out is not None:
            return x, mask_out
        return x


class PartialConv2dBlock(_BasePartialConvBlock):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, padding_mode='zeros', weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, nonlinearity='none', inplace_nonlinearity=False,
                 multi_channel=False, return_mask=True, apply_noise=False, order='CNA'):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation,
                         groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, nonlinearity,
                         inplace_nonlinearity, multi_channel, return_mask, apply_noise, order,
                         2)


class PartialConv3dBlock(_BasePartialConvBlock):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, padding_mode='zeros', weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, nonlinearity='none', inplace_nonlinearity=False,
                 multi_channel=False, return_mask=True, apply_noise=False, order='CNA'):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation,
                         groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, nonlinearity,
                         inplace_nonlinearity, multi_channel, return_mask, apply_noise, order,
                         3)


class _MultiOutBaseConvBlock(_BaseConvBlock):
    """Block whose layers may return auxiliary outputs (conv.py:806-848)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, dilation,
                 groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                 activation_norm_type, activation_norm_params, nonlinearity,
                 inplace_nonlinearity, apply_noise, order, input_dim):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation,
                         groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, nonlinearity,
                         inplace_nonlinearity, apply_noise, order, input_dim)
        self.multiple_outputs = True

    def forward(self, x, *cond_inputs, **kw_cond_inputs):
        other_outputs = []
        for layer in self.layers.values():
            if getattr(layer, 'conditional', False):
                x = layer(x, *cond_inputs, **kw_cond_inputs)
            if getattr(layer, 'multiple_outputs', False):
                x, other_output = layer(x)
                other_outputs.append(other_output)
            else:
                x = layer(x)
        return (x, *other_outputs)


class MultiOutConv2dBlock(_MultiOutBaseConvBlock):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, padding_mode='zeros', weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, nonlinearity='none', inplace_nonlinearity=False,
                 apply_noise=False, order='CNA'):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation,
                         groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, nonlinearity,
                         inplace_nonlinearity, apply_noise, order, 2)


class NHWCConv2d(nn.Conv2d):
    """``nn.Conv2d`` (same parameters and state-dict keys) that runs through the k10 / k11 conv
    routing of :mod:`imaginaire_amd.ops.conv` instead of calling MIOpen directly — the bare
    1x1 style heads of the MUNIT / FUNIT style encoders (reference generators/munit.py:
    ``nn.Conv2d(num_filters, style_channels, 1, 1, 0)``); inside a captured graph MIOpen's
    small-problem backward solvers must not run."""

    def forward(self, x):
        return nhwc_conv.conv2d(x, self.weight, self.bias, self.stride, self.padding,
                                self.dilation, self.groups, self.padding_mode)


class PartialConv2d(nn.Conv2d):
    """Partial convolution (Liu et al.; reference conv.py:927-1009).

    The masked convolution runs on MIOpen without bias; the mask window sums,
    the ``winsize/(sum+eps)`` re-normalisation, bias re-add and mask multiply
    run in one HIP kernel (k3, ops/partial_conv.py).
    """

    def __init__(self, *args, multi_channel=False, return_mask=True, **kwargs):
        self.multi_channel = multi_channel
        self.return_mask = return_mask
        super().__init__(*args, **kwargs)
        k0, k1 = self.kernel_size
        self.slide_winsize = (self.in_channels if multi_channel else 1) * k0 * k1
        self.partial_conv = True

    def forward(self, x, mask_in=None):
        assert x.dim() == 4
        if mask_in is None:
            shape = (x.shape[0], x.shape[1] if self.multi_channel else 1, x.shape[2], x.shape[3])
            mask = torch.ones(shape, device=x.device, dtype=x.dtype)
            xin = x
        else:
            mask = mask_in
            xin = x * mask
            if self.multi_channel and mask.shape[1] == 1 and self.in_channels > 1:
                mask = mask.expand(-1, self.in_channels, -1, -1)
        raw = nhwc_conv.conv2d(xin, self.weight, None, self.stride, self.padding, self.dilation,
                       self.groups)
        out, update_mask = partial_conv_renorm(raw, mask, self.bias, self.kernel_size,
                                               self.stride, self.padding, self.dilation,
                                               self.slide_winsize, eps=1e-6)
        if self.multi_channel:
            update_mask = update_mask.expand(-1, self.out_channels, -1, -1)
        if self.return_mask:
            return out, update_mask
        return out


class PartialConv3d(nn.Conv3d):
    """3-D partial convolution (reference conv.py:1012-1072)."""

    def __init__(self, *args, multi_channel=False, return_mask=True, **kwargs):
        self.multi_channel = multi_channel
        self.return_mask = return_mask
        super().__init__(*args, **kwargs)
        if self.multi_channel:
            w = torch.ones(self.out_channels, self.in_channels, *self.kernel_size)
        else:
            w = torch.ones(1, 1, *self.kernel_size)
        self.register_buffer('weight_maskUpdater', w, persistent=False)
        self.slide_winsize = w.shape[1] * w.shape[2] * w.shape[3] * w.shape[4]
        self.partial_conv = True

    def forward(self, x, mask_in=None):
        assert x.dim() == 5
        with torch.no_grad():
            update_mask = F.conv3d(mask_in, self.weight_maskUpdater.to(mask_in), bias=None,
                                   stride=self.stride, padding=self.padding,
                                   dilation=self.dilation, groups=1)
            mask_ratio = self.slide_winsize / (update_mask + 1e-8)
            update_mask = torch.clamp(update_mask, 0, 1)
            mask_ratio = torch.mul(mask_ratio, update_mask)
        raw_out = super().forward(torch.mul(x, mask_in))
        if self.bias is not None:
            bias_view = self.bias.view(1, self.out_channels, 1, 1, 1)
            output = torch.mul(raw_out - bias_view, mask_ratio) + bias_view
            if mask_in is not None:
                output = torch.mul(output, update_mask)
        else:
            output = torch.mul(raw_out, mask_ratio)
        if self.return_mask:
            return output, update_mask
        return output
