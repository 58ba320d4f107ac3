"""Residual blocks (reference layers/residual.py:16-1235).

Same module names (``conv_block_0/1/s``), the same ``order`` semantics
(``'pre_act'`` → ``'NACNAC'``), learned 1×1 shortcut when in≠out, bias list
``[b0, b1, bs]`` and optional activation checkpointing of the residual branch.
The blocks' norm/activation pairs run as fused HIP kernels via the conv blocks.
"""
import functools

from torch import nn
from imaginaire_amd.ops.pool import AvgPool2d
from imaginaire_amd.ops.resize import Upsample as NearestUpsample
from torch.utils.checkpoint import checkpoint

from .conv import (Conv1dBlock, Conv2dBlock, Conv3dBlock, HyperConv2dBlock, LinearBlock,
                   MultiOutConv2dBlock, PartialConv2dBlock, PartialConv3dBlock, _BaseConvBlock)


class _BaseResBlock(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                 padding_mode, weight_norm_type, weight_norm_params, activation_norm_type,
                 activation_norm_params, skip_activation_norm, skip_nonlinearity, nonlinearity,
                 inplace_nonlinearity, apply_noise, hidden_channels_equal_out_channels, order,
                 block, learn_shortcut):
        super().__init__()
        if order == 'pre_act':
            order = 'NACNAC'
        if isinstance(bias, bool):
            biases = [bias, bias, bias]
        elif isinstance(bias, list):
            if len(bias) != 3:
                raise ValueError('Bias list must be 3.')
            biases = bias
        else:
            raise ValueError('Bias must be either an integer or s list.')
        self.learn_shortcut = (in_channels != out_channels) or learn_shortcut
        if len(order) > 6 or len(order) < 5:
            raise ValueError('order must be either 5 or 6 characters')
        hidden_channels = out_channels if hidden_channels_equal_out_channels \
            else min(in_channels, out_channels)
        conv_main_params = {}
        conv_skip_params = {}
        if block != LinearBlock:
            conv_base_params = dict(stride=1, dilation=dilation, groups=groups,
                                    padding_mode=padding_mode)
            conv_main_params.update(conv_base_params)
            conv_main_params.update(dict(kernel_size=kernel_size,
                                         activation_norm_type=activation_norm_type,
                                         activation_norm_params=activation_norm_params,
                                         padding=padding))
            conv_skip_params.update(conv_base_params)
            conv_skip_params.update(dict(kernel_size=1))
            if skip_activation_norm:
                conv_skip_params.update(dict(activation_norm_type=activation_norm_type,
                                             activation_norm_params=activation_norm_params))
        other_params = dict(weight_norm_type=weight_norm_type,
                            weight_norm_params=weight_norm_params, apply_noise=apply_noise)
        if order.find('A') < order.find('C') and \
                (activation_norm_type == '' or activation_norm_type == 'none'):
            first_inplace = False
        else:
            first_inplace = inplace_nonlinearity
        self.conv_block_0 = block(in_channels, hidden_channels, bias=biases[0],
                                  nonlinearity=nonlinearity, order=order[0:3],
                                  inplace_nonlinearity=first_inplace, **conv_main_params,
                                  **other_params)
        self.conv_block_1 = block(hidden_channels, out_channels, bias=biases[1],
                                  nonlinearity=nonlinearity, order=order[3:],
                                  inplace_nonlinearity=inplace_nonlinearity, **conv_main_params,
                                  **other_params)
        if self.learn_shortcut:
            skip_nonlinearity_type = nonlinearity if skip_nonlinearity else ''
            self.conv_block_s = block(in_channels, out_channels, bias=biases[2],
                                      nonlinearity=skip_nonlinearity_type, order=order[0:3],
                                      **conv_skip_params, **other_params)
        self.conditional = getattr(self.conv_block_0, 'conditional', False) or \
            getattr(self.conv_block_1, 'conditional', False)

    def conv_blocks(self, x, *cond_inputs, **kw_cond_inputs):
        dx = self.conv_block_0(x, *cond_inputs, **kw_cond_inputs)
        dx = self.conv_block_1(dx, *cond_inputs, **kw_cond_inputs)
        return dx

    def _fused_shortcut_ok(self):
        """The shortcut can be added inside conv_block_1 (its epilogue when it ends in a conv):
        a plain conv block, and no noise layer in conv_block_1 / conv_block_s, whose random
        draws would change order (the reference computes the branch before the shortcut)."""
        ok = getattr(self, '_fuse_ok', None)
        if ok is None:
            ok = type(self.conv_block_1).forward is _BaseConvBlock.forward and \
                'noise' not in self.conv_block_1.layers and \
                not (self.learn_shortcut and 'noise' in getattr(self.conv_block_s, 'layers', {}))
            self._fuse_ok = ok
        return ok

    def forward(self, x, *cond_inputs, do_checkpoint=False, **kw_cond_inputs):
        if not do_checkpoint and self._fused_shortcut_ok():
            # x_shortcut + dx with the add in the epilogue of the branch's last conv (k10) when
            # the branch ends in one (pre-activation 'NACNAC' blocks of SPADE / FUNIT / the
            # residual discriminators): one full-tensor pass fewer per block
            dx = self.conv_block_0(x, *cond_inputs, **kw_cond_inputs)
            if self.learn_shortcut:
                x_shortcut = self.conv_block_s(x, *cond_inputs, **kw_cond_inputs)
            else:
                x_shortcut = x
            return self.conv_block_1(dx, *cond_inputs, residual=x_shortcut, **kw_cond_inputs)
        if do_checkpoint:
            dx = checkpoint(self.conv_blocks, x, *cond_inputs, use_reentrant=False,
                            **kw_cond_inputs)
        else:
            dx = self.conv_blocks(x, *cond_inputs, **kw_cond_inputs)
        if self.learn_shortcut:
            x_shortcut = self.conv_block_s(x, *cond_inputs, **kw_cond_inputs)
        else:
            x_shortcut = x
        return x_shortcut + dx


def _res_init(block_cls):
    def __init__(self, in_channels, out_channels, kernel_size=3, padding=1, dilation=1,
                 groups=1, bias=True, padding_mode='zeros', weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, skip_activation_norm=True,
                 skip_nonlinearity=False, nonlinearity='leakyrelu', inplace_nonlinearity=False,
                 apply_noise=False, hidden_channels_equal_out_channels=False, order='CNACNA',
                 learn_shortcut=False):
        _BaseResBlock.__init__(self, in_channels, out_channels, kernel_size, padding, dilation,
                               groups, bias, padding_mode, weight_norm_type, weight_norm_params,
                               activation_norm_type, activation_norm_params,
                               skip_activation_norm, skip_nonlinearity, nonlinearity,
                               inplace_nonlinearity, apply_noise,
                               hidden_channels_equal_out_channels, order, block_cls,
                               learn_shortcut)
    return __init__


class ResLinearBlock(_BaseResBlock):
    def __init__(self, in_channels, out_channels, bias=True, weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, skip_activation_norm=True,
                 skip_nonlinearity=False, nonlinearity='leakyrelu', inplace_nonlinearity=False,
                 apply_noise=False, hidden_channels_equal_out_channels=False, order='CNACNA',
                 learn_shortcut=False):
        super().__init__(in_channels, out_channels, None, None, None, None, bias, None,
                         weight_norm_type, weight_norm_params, activation_norm_type,
                         activation_norm_params, skip_activation_norm, skip_nonlinearity,
                         nonlinearity, inplace_nonlinearity, apply_noise,
                         hidden_channels_equal_out_channels, order, LinearBlock,
                         learn_shortcut)


class Res1dBlock(_BaseResBlock):
    __init__ = _res_init(Conv1dBlock)


class Res2dBlock(_BaseResBlock):
    __init__ = _res_init(Conv2dBlock)


class Res3dBlock(_BaseResBlock):
    __init__ = _res_init(Conv3dBlock)


class _BaseHyperResBlock(_BaseResBlock):
    def __init__(self, in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                 padding_mode, weight_norm_type, weight_norm_params, activation_norm_type,
                 activation_norm_params, skip_activation_norm, skip_nonlinearity, nonlinearity,
                 inplace_nonlinearity, apply_noise, hidden_channels_equal_out_channels, order,
                 is_hyper_conv, is_hyper_norm, block, learn_shortcut):
        block = functools.partial(block, is_hyper_conv=is_hyper_conv, is_hyper_norm=is_hyper_norm)
        super().__init__(in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                         padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, skip_activation_norm,
                         skip_nonlinearity, nonlinearity, inplace_nonlinearity, apply_noise,
                         hidden_channels_equal_out_channels, order, block, learn_shortcut)

    def forward(self, x, *cond_inputs, conv_weights=(None,) * 3, norm_weights=(None,) * 3,
                **kw_cond_inputs):
        dx = self.conv_block_0(x, *cond_inputs, conv_weights=conv_weights[0],
                               norm_weights=norm_weights[0])
        dx = self.conv_block_1(dx, *cond_inputs, conv_weights=conv_weights[1],
                               norm_weights=norm_weights[1])
        if self.learn_shortcut:
            x_shortcut = self.conv_block_s(x, *cond_inputs, conv_weights=conv_weights[2],
                                           norm_weights=norm_weights[2])
        else:
            x_shortcut = x
        return x_shortcut + dx


class HyperRes2dBlock(_BaseHyperResBlock):
    def __init__(self, in_channels, out_channels, kernel_size=3, padding=1, dilation=1,
                 groups=1, bias=True, padding_mode='zeros', weight_norm_type='',
                 weight_norm_params=None, activation_norm_type='', activation_norm_params=None,
                 skip_activation_norm=True, skip_nonlinearity=False, nonlinearity='leakyrelu',
                 inplace_nonlinearity=False, apply_noise=False,
                 hidden_channels_equal_out_channels=False, order='CNACNA', is_hyper_conv=False,
                 is_hyper_norm=False, learn_shortcut=False):
        super().__init__(in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                         padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, skip_activation_norm,
                         skip_nonlinearity, nonlinearity, inplace_nonlinearity, apply_noise,
                         hidden_channels_equal_out_channels, order, is_hyper_conv,
                         is_hyper_norm, HyperConv2dBlock, learn_shortcut)


class _BaseDownResBlock(_BaseResBlock):
    def __init__(self, in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                 padding_mode, weight_norm_type, weight_norm_params, activation_norm_type,
                 activation_norm_params, skip_activation_norm, skip_nonlinearity, nonlinearity,
                 inplace_nonlinearity, apply_noise, hidden_channels_equal_out_channels, order,
                 block, pooling, down_factor, learn_shortcut):
        super().__init__(in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                         padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, skip_activation_norm,
                         skip_nonlinearity, nonlinearity, inplace_nonlinearity, apply_noise,
                         hidden_channels_equal_out_channels, order, block, learn_shortcut)
        self.pooling = pooling(down_factor)

    def forward(self, x, *cond_inputs):
        dx = self.conv_block_0(x, *cond_inputs)
        dx = self.conv_block_1(dx, *cond_inputs)
        dx = self.pooling(dx)
        x_shortcut = self.conv_block_s(x, *cond_inputs) if self.learn_shortcut else x
        return self.pooling(x_shortcut) + dx


class DownRes2dBlock(_BaseDownResBlock):
    def __init__(self, in_channels, out_channels, kernel_size=3, padding=1, dilation=1,
                 groups=1, bias=True, padding_mode='zeros', weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, skip_activation_norm=True,
                 skip_nonlinearity=False, nonlinearity='leakyrelu', inplace_nonlinearity=False,
                 apply_noise=False, hidden_channels_equal_out_channels=False, order='CNACNA',
                 pooling=AvgPool2d, down_factor=2, learn_shortcut=False):
        super().__init__(in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                         padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, skip_activation_norm,
                         skip_nonlinearity, nonlinearity, inplace_nonlinearity, apply_noise,
                         hidden_channels_equal_out_channels, order, Conv2dBlock, pooling,
                         down_factor, learn_shortcut)


class _BaseUpResBlock(_BaseResBlock):
    def __init__(self, in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                 padding_mode, weight_norm_type, weight_norm_params, activation_norm_type,
                 activation_norm_params, skip_activation_norm, skip_nonlinearity, nonlinearity,
                 inplace_nonlinearity, apply_noise, hidden_channels_equal_out_channels, order,
                 block, upsample, up_factor, learn_shortcut):
        super().__init__(in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                         padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, skip_activation_norm,
                         skip_nonlinearity, nonlinearity, inplace_nonlinearity, apply_noise,
                         hidden_channels_equal_out_channels, order, block, learn_shortcut)
        self.order = order
        self.upsample = upsample(scale_factor=up_factor)

    def forward(self, x, *cond_inputs):
        x_shortcut = self.upsample(x)
        if self.learn_shortcut:
            x_shortcut = self.conv_block_s(x_shortcut, *cond_inputs)
        if self.order[0:3] == 'NAC':
            # norm + act at low resolution, upsample, then conv (residual.py:779-786)
            layers = self.conv_block_0.layers
            norm = layers['norm'] if 'norm' in layers else None
            act = layers['nonlinearity'] if 'nonlinearity' in layers else None
            from .nonlinearity import act_slope
            slope = act_slope(act)
            if norm is not None and getattr(norm, 'supports_fused_act', False) and \
                    slope is not None:
                if getattr(norm, 'conditional', False):
                    x = norm(x, *cond_inputs, act_slope=slope)
                else:
                    x = norm(x, act_slope=slope)
                x = self.upsample(x)
                x = layers['conv'](x)
            else:
                for ix, layer in enumerate(layers.values()):
                    if getattr(layer, 'conditional', False):
                        x = layer(x, *cond_inputs)
                    else:
                        x = layer(x)
                    if ix == 1:
                        x = self.upsample(x)
        else:
            x = self.conv_block_0(x, *cond_inputs)
            x = self.upsample(x)
        x = self.conv_block_1(x, *cond_inputs)
        return x_shortcut + x


class UpRes2dBlock(_BaseUpResBlock):
    def __init__(self, in_channels, out_channels, kernel_size=3, padding=1, dilation=1,
                 groups=1, bias=True, padding_mode='zeros', weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, skip_activation_norm=True,
                 skip_nonlinearity=False, nonlinearity='leakyrelu', inplace_nonlinearity=False,
                 apply_noise=False, hidden_channels_equal_out_channels=False, order='CNACNA',
                 upsample=NearestUpsample, up_factor=2, learn_shortcut=False):
        super().__init__(in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                         padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, skip_activation_norm,
                         skip_nonlinearity, nonlinearity, inplace_nonlinearity, apply_noise,
                         hidden_channels_equal_out_channels, order, Conv2dBlock, upsample,
                         up_factor, learn_shortcut)


class _BasePartialResBlock(_BaseResBlock):
    def __init__(self, in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                 padding_mode, weight_norm_type, weight_norm_params, activation_norm_type,
                 activation_norm_params, skip_activation_norm, skip_nonlinearity, nonlinearity,
                 inplace_nonlinearity, multi_channel, return_mask, apply_noise,
                 hidden_channels_equal_out_channels, order, block, learn_shortcut):
        block = functools.partial(block, multi_channel=multi_channel, return_mask=return_mask)
        self.partial_conv = True
        super().__init__(in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                         padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, skip_activation_norm,
                         skip_nonlinearity, nonlinearity, inplace_nonlinearity, apply_noise,
                         hidden_channels_equal_out_channels, order, block, learn_shortcut)

    def forward(self, x, *cond_inputs, mask_in=None, **kw_cond_inputs):
        if self.conv_block_0.layers.conv.return_mask:
            dx, mask_out = self.conv_block_0(x, *cond_inputs, mask_in=mask_in, **kw_cond_inputs)
            dx, mask_out = self.conv_block_1(dx, *cond_inputs, mask_in=mask_out,
                                             **kw_cond_inputs)
        else:
            dx = self.conv_block_0(x, *cond_inputs, mask_in=mask_in, **kw_cond_inputs)
            dx = self.conv_block_1(dx, *cond_inputs, mask_in=mask_in, **kw_cond_inputs)
            mask_out = None
        if self.learn_shortcut:
            x_shortcut = self.conv_block_s(x, *cond_inputs, mask_in=mask_in, **kw_cond_inputs)
            if type(x_shortcut) == tuple:
                x_shortcut, _ = x_shortcut
        else:
            x_shortcut = x
        output = x_shortcut + dx
        if mask_out is not None:
            return output, mask_out
        return output


def _partial_res_init(block_cls):
    def __init__(self, in_channels, out_channels, kernel_size=3, padding=1, dilation=1,
                 groups=1, bias=True, padding_mode='zeros', weight_norm_type='none',
                 weight_norm_params=None, activation_norm_type='none',
                 activation_norm_params=None, skip_activation_norm=True,
                 skip_nonlinearity=False, nonlinearity='leakyrelu', inplace_nonlinearity=False,
                 multi_channel=False, return_mask=True, apply_noise=False,
                 hidden_channels_equal_out_channels=False, order='CNACNA',
                 learn_shortcut=False):
        _BasePartialResBlock.__init__(self, in_channels, out_channels, kernel_size, padding,
                                      dilation, groups, bias, padding_mode, weight_norm_type,
                                      weight_norm_params, activation_norm_type,
                                      activation_norm_params, skip_activation_norm,
                                      skip_nonlinearity, nonlinearity, inplace_nonlinearity,
                                      multi_channel, return_mask, apply_noise,
                                      hidden_channels_equal_out_channels, order, block_cls,
                                      learn_shortcut)
    return __init__


class PartialRes2dBlock(_BasePartialResBlock):
    __init__ = _partial_res_init(PartialConv2dBlock)


class PartialRes3dBlock(_BasePartialResBlock):
    __init__ = _partial_res_init(PartialConv3dBlock)


class _BaseMultiOutResBlock(_BaseResBlock):
    def __init__(self, in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                 padding_mode, weight_norm_type, weight_norm_params, activation_norm_type,
                 activation_norm_params, skip_activation_norm, skip_nonlinearity, nonlinearity,
                 inplace_nonlinearity, apply_noise, hidden_channels_equal_out_channels, order,
                 block, learn_shortcut):
        self.multiple_outputs = True
        super().__init__(in_channels, out_channels, kernel_size, padding, dilation, groups, bias,
                         padding_mode, weight_norm_type, weight_norm_params,
                         activation_norm_type, activation_norm_params, skip_activation_norm,
                         skip_nonlinearity, nonlinearity, inplace_nonlinearity, apply_noise,
                         hidden_channels_equal_out_channels, order, block, learn_shortcut)

    def forward(self, x, *cond_inputs):
        dx, aux_outputs_0 = self.conv_block_0(x, *cond_inputs)
        dx, aux_outputs_1 = self.conv_block_1(dx, *cond_inputs)
        if self.learn_shortcut:
            x_shortcut, _ = self.conv_block_s(x, *cond_inputs)
        else:
            x_shortcut = x
        return x_shortcut + dx, aux_outputs_0, aux_outputs_1


class MultiOutRes2dBlock(_BaseMultiOutResBlock):
    def __init__(self, *args, **kwargs):
        _res_init(MultiOutConv2dBlock)(self, *args, **kwargs)
        self.multiple_outputs = True
