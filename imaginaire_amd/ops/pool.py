"""NHWC average pooling (k14, ``csrc/pool.hip``) with a gather backward, and NHWC max pooling
over non-overlapping windows (``max_pool2d``).

``avg_pool2d`` / ``AvgPool2d`` are drop-ins for ``F.avg_pool2d`` / ``nn.AvgPool2d`` (no
parameters, identical state dicts). Packed channels-last bf16 / fp32 activations run the HIP
kernels (16-byte accesses when the channel count divides by 8, per-channel otherwise: the
185-channel COCO-Stuff label maps); anything else (CPU, NCHW, ``ceil_mode``,
``divisor_override``) falls back to PyTorch.
"""
import torch
import torch.nn.functional as F
from torch import nn

from imaginaire_amd.ops import _ext


def _pair(v):
    return (int(v), int(v)) if not isinstance(v, (tuple, list)) else (int(v[0]), int(v[1]))


class _AvgPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, include_pad):
        ctx.conf = (x.shape[2], x.shape[3], k, s, p, include_pad)
        return _ext.ext().avg_pool_nhwc_fwd(x, k[0], k[1], s[0], s[1], p[0], p[1], include_pad)

    @staticmethod
    def backward(ctx, dy):
        h, w, k, s, p, include_pad = ctx.conf
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = _ext.ext().avg_pool_nhwc_bwd(dy, h, w, k[0], k[1], s[0], s[1], p[0], p[1],
                                          include_pad)
        return dx, None, None, None, None


def avg_pool2d(x, kernel_size, stride=None, padding=0, ceil_mode=False, count_include_pad=True,
               divisor_override=None):
    k = _pair(kernel_size)
    s = _pair(stride if stride is not None else kernel_size)
    p = _pair(padding)
    if x.is_cuda and x.dim() == 4 and not ceil_mode and divisor_override is None and \
            x.dtype in (torch.bfloat16, torch.float32) and \
            x.is_contiguous(memory_format=torch.channels_last) and _ext.use_native(x) and \
            2 * p[0] <= k[0] and 2 * p[1] <= k[1] and \
            x.shape[2] + 2 * p[0] >= k[0] and x.shape[3] + 2 * p[1] >= k[1]:
        y = _AvgPoolNHWC.apply(x, k, s, p, bool(count_include_pad))
    else:
        y = F.avg_pool2d(x, kernel_size, stride, padding, ceil_mode, count_include_pad,
                         divisor_override)
    valid = getattr(x, '_iamd_valid_channels', None)
    if valid is not None:  # pooling acts per channel: a zero channel tail stays zero
        y._iamd_valid_channels = valid
    return y


class _MaxPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k):
        ctx.k = k
        ctx.save_for_backward(x)
        return _ext.ext().max_pool_nhwc_fwd(x, k[0], k[1])

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        if dy.dtype != x.dtype:
            dy = dy.to(x.dtype)
        return _ext.ext().max_pool_nhwc_bwd(x, dy, ctx.k[0], ctx.k[1]), None


def max_pool2d(x, kernel_size, stride=None, padding=0, dilation=1, ceil_mode=False,
               return_indices=False):
    """``F.max_pool2d``. Non-overlapping windows (kernel == stride, no padding / dilation — VGG's
    2x2 pools) on packed NHWC bf16 / fp32 activations run the k14 max-pool kernels (the backward
    recomputes each window's argmax from the input: no int64 index tensor); anything else runs
    PyTorch."""
    k = _pair(kernel_size)
    s = _pair(stride if stride is not None else kernel_size)
    if x.is_cuda and x.dim() == 4 and k == s and _pair(padding) == (0, 0) and \
            _pair(dilation) == (1, 1) and not ceil_mode and not return_indices and \
            x.dtype in (torch.bfloat16, torch.float32) and \
            x.is_contiguous(memory_format=torch.channels_last) and _ext.use_native(x) and \
            x.shape[2] >= k[0] and x.shape[3] >= k[1]:
        return _MaxPoolNHWC.apply(x, k)
    return F.max_pool2d(x, kernel_size, stride, padding, dilation, ceil_mode, return_indices)


class AvgPool2d(nn.Module):
    """Drop-in for ``nn.AvgPool2d`` running k14 on NHWC activations."""

    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False,
                 count_include_pad=True, divisor_override=None):
        super().__init__()
        self.kernel_size = kernel_size
        self.stride = stride if stride is not None else kernel_size
        self.padding = padding
        self.ceil_mode = ceil_mode
        self.count_include_pad = count_include_pad
        self.divisor_override = divisor_override

    def forward(self, x):
        return avg_pool2d(x, self.kernel_size, self.stride, self.padding, self.ceil_mode,
                          self.count_include_pad, self.divisor_override)

    def extra_repr(self):
        return 'kernel_size={}, stride={}, padding={}'.format(self.kernel_size, self.stride,
                                                              self.padding)


class ReflectionPad2d(nn.Module):
    """Drop-in for ``nn.ReflectionPad2d`` running the NHWC gather kernels forward and backward
    (ops/conv.py ``pad``; PyTorch's reflection-pad backward scatters with atomics, and its
    output drops the channels-last layout the following pooling kernel needs)."""

    def __init__(self, padding):
        super().__init__()
        self.padding = (padding,) * 4 if isinstance(padding, int) else tuple(padding)

    def forward(self, x):
        from imaginaire_amd.ops.conv import nhwc, pad
        if x.is_cuda and x.dim() == 4:
            x = nhwc(x)
        return pad(x, self.padding, 'reflect')

    def extra_repr(self):
        return str(self.padding)

