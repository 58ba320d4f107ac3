"""Resampling that keeps the activation dtype under bf16 autocast.

torch.autocast runs ``upsample_*`` in fp32: every nearest/bilinear resize of a bf16 activation
becomes bf16->fp32 cast + fp32 resize + an fp32 tensor that the next fused norm kernel then
reads at twice the bytes (measured on MI355X: ~800 bf16->fp32 copy launches and fp32
``apply_fwd`` norm kernels per 3 SPADE steps, profiles/spade_step_k11v2_mi355x.txt). Nearest
resizing is exact in any dtype, so it runs on the input dtype with autocast disabled
instead. Bilinear resizes of packed NHWC activations (channels % 8 == 0) run the k12 HIP
kernel (``csrc/resize.hip``) in the activation dtype with a deterministic gather backward.
Used by every resize on the SPADE/pix2pixHD/vid2vid paths (reference: plain
``F.interpolate`` / ``nn.Upsample``).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from imaginaire_amd.ops import _ext


def _pair(v):
    return (v, v) if not isinstance(v, (tuple, list)) else tuple(v)


def _src_scale(n_in, n_out, align_corners, sf):
    """PyTorch's area_pixel_compute_scale (float32 like its accscalar)."""
    if align_corners:
        return float(np.float32(n_in - 1) / np.float32(n_out - 1)) if n_out > 1 else 0.0
    if sf is not None and sf > 0:
        return 1.0 / sf
    return n_in / n_out


class _BilinearNHWC(torch.autograd.Function):
    """k12 bilinear resize (+ optional fused residual add); gather-form backward."""

    @staticmethod
    def forward(ctx, x, add, ho, wo, sh, sw, ac):
        y = _ext.ext().resize_bilinear_fwd(x, ho, wo, sh, sw, ac, add)
        ctx.conf = (x.shape[2], x.shape[3], sh, sw, ac, add is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        h, w, sh, sw, ac, has_add = ctx.conf
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = _ext.ext().resize_bilinear_bwd(dy, h, w, sh, sw, ac) \
            if ctx.needs_input_grad[0] else None
        return dx, (dy if has_add and ctx.needs_input_grad[1] else None), \
            None, None, None, None, None


class _NearestNHWC(torch.autograd.Function):
    """k12 nearest resize (16-byte gathers in the activation dtype); gather-form backward."""

    @staticmethod
    def forward(ctx, x, ho, wo, sh, sw):
        ctx.conf = (x.shape[2], x.shape[3], sh, sw)
        return _ext.ext().resize_nearest_fwd(x, ho, wo, sh, sw)

    @staticmethod
    def backward(ctx, dy):
        h, w, sh, sw = ctx.conf
        dy = dy.contiguous(memory_format=torch.channels_last)
        return _ext.ext().resize_nearest_bwd(dy, h, w, sh, sw), None, None, None, None


def _nearest(x, size, scale_factor):
    h, w = x.shape[2], x.shape[3]
    sfh, sfw = _pair(scale_factor) if scale_factor is not None else (None, None)
    if size is not None:
        ho, wo = _pair(size)
        sfh = sfw = None
    else:
        ho, wo = int(math.floor(h * sfh)), int(math.floor(w * sfw))
    # the backward's gather lists cover up to 5x upsampling per axis
    if ho > 5 * h or wo > 5 * w:
        return None
    return _NearestNHWC.apply(x, ho, wo, _src_scale(h, ho, False, sfh),
                              _src_scale(w, wo, False, sfw))


def _bilinear_native_ok(x):
    return x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float32) and \
        x.shape[1] % 8 == 0 and x.is_contiguous(memory_format=torch.channels_last) and \
        _ext.use_native(x)


def _bilinear(x, size, scale_factor, align_corners, add=None):
    h, w = x.shape[2], x.shape[3]
    sfh, sfw = _pair(scale_factor) if scale_factor is not None else (None, None)
    if size is not None:
        ho, wo = _pair(size)
        sfh = sfw = None
    else:
        ho, wo = int(math.floor(h * sfh)), int(math.floor(w * sfw))
    ac = bool(align_corners)
    y = _BilinearNHWC.apply(x, add, ho, wo, _src_scale(h, ho, ac, sfh),
                            _src_scale(w, wo, ac, sfw), ac)
    valid = getattr(x, '_iamd_valid_channels', None)
    if valid is not None:  # zero channel tail stays zero
        y._iamd_valid_channels = valid
    return y


def upsample_add(x, add, scale_factor=2, align_corners=False):
    """``F.interpolate(x, scale_factor, 'bilinear', align_corners) + add`` — one k12 pass on
    the GPU (reference FPSE top-down path, discriminators/fpse.py:74-101)."""
    if _bilinear_native_ok(x) and add.shape[1] == x.shape[1]:
        add = add.to(x.dtype).contiguous(memory_format=torch.channels_last)
        return _bilinear(x, None, scale_factor, align_corners, add)
    return interpolate(x, scale_factor=scale_factor, mode='bilinear',
                       align_corners=align_corners) + add


def interpolate(x, size=None, scale_factor=None, mode='nearest', align_corners=None,
                recompute_scale_factor=None):
    # bilinear on NHWC activations: the k12 kernel in the activation dtype (autocast would
    # run an fp32 resize whose backward is an atomic scatter)
    if recompute_scale_factor and scale_factor is not None and size is None and \
            _bilinear_native_ok(x) and mode in ('bilinear', 'nearest'):
        # recomputed scale = in / out of the floored size: the same as passing the size
        sfh, sfw = _pair(scale_factor)
        size = (int(math.floor(x.shape[2] * sfh)), int(math.floor(x.shape[3] * sfw)))
        scale_factor, recompute_scale_factor = None, None
    if mode == 'bilinear' and not recompute_scale_factor and _bilinear_native_ok(x):
        return _bilinear(x, size, scale_factor, align_corners)
    if mode == 'nearest' and not recompute_scale_factor and _bilinear_native_ok(x):
        y = _nearest(x, size, scale_factor)
        if y is not None:
            valid = getattr(x, '_iamd_valid_channels', None)
            if valid is not None:
                y._iamd_valid_channels = valid
            return y
    if mode == 'nearest' and x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and \
            torch.is_autocast_enabled('cuda'):
        with torch.autocast('cuda', enabled=False):
            y = F.interpolate(x, size, scale_factor, mode, align_corners,
                              recompute_scale_factor)
    else:
        y = F.interpolate(x, size, scale_factor, mode, align_corners, recompute_scale_factor)
    valid = getattr(x, '_iamd_valid_channels', None)
    if valid is not None:  # resizes act per channel: a zero channel tail stays zero
        y._iamd_valid_channels = valid
    return y


class Upsample(nn.Module):
    """Drop-in for ``nn.Upsample`` (no parameters, identical state dict)."""

    def __init__(self, size=None, scale_factor=None, mode='nearest', align_corners=None):
        super().__init__()
        self.size = size
        self.scale_factor = float(scale_factor) if scale_factor else None
        self.mode = mode
        self.align_corners = align_corners

    def forward(self, x):
        return interpolate(x, self.size, self.scale_factor, self.mode, self.align_corners)

    def extra_repr(self):
        return 'scale_factor={}, mode={}'.format(self.scale_factor, self.mode)
