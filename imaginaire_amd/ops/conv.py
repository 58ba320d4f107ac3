"""NHWC convolution entry points.

MIOpen's fast NHWC solvers (igemm / CK xdlops) require *packed* NHWC
activations AND weights. When the two layouts differ (e.g. an NCHW-strided
weight against a channels-last activation, or the NCHW output of a
reflection pad), MIOpen falls back to its naive direct kernels — measured
at >95% of a SPADE step on MI355X before this helper existed
(profiles/spade_step_naive_conv_mi355x.txt). Every convolution issued by
the framework's layers goes through here so both operands are packed
channels-last on the GPU (a no-op when they already are).
"""
import torch
import torch.nn.functional as F

_CL = torch.channels_last


def nhwc(t):
    """Packed channels-last view/copy of a 4-D CUDA tensor (identity otherwise)."""
    if t is not None and t.is_cuda and t.dim() == 4 and not t.is_contiguous(memory_format=_CL):
        return t.contiguous(memory_format=_CL)
    return t


def _pad_arg(padding):
    if isinstance(padding, int):
        return [padding] * 4
    ph, pw = padding
    return [pw, pw, ph, ph]


def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1,
           padding_mode='zeros'):
    if padding_mode != 'zeros' and padding_mode is not None:
        x = F.pad(x, _pad_arg(padding), mode=padding_mode)
        padding = 0
    if x.is_cuda:
        x = nhwc(x)
        weight = nhwc(weight)
    return F.conv2d(x, weight, bias, stride, padding, dilation, groups)


def conv_transpose2d(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1,
                     dilation=1):
    if x.is_cuda:
        x = nhwc(x)
        weight = nhwc(weight)
    return F.conv_transpose2d(x, weight, bias, stride, padding, output_padding, groups, dilation)
