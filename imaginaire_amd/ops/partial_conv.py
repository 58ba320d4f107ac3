"""Partial-convolution re-normalisation (k3, ``csrc/partial_conv.hip``).

``partial_conv_renorm(raw, mask, bias, ...)`` takes the *bias-free* output of
``conv(x * mask)`` and returns ``(out, update_mask)`` with the semantics of the
reference PartialConv2d (layers/conv.py:956-1009)::

    s = conv(mask, ones); update = clamp(s, 0, 1)
    out = (raw * winsize / (s + eps) * update + bias) * update

The mask is treated as a constant (reference computes it under ``no_grad``).
"""
import torch
import torch.nn.functional as F

from imaginaire_amd.ops import _ext


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def _mask_stats_reference(mask, kernel_size, stride, padding, dilation, winsize, eps):
    kh, kw = _pair(kernel_size)
    ones = torch.ones(1, mask.shape[1], kh, kw, device=mask.device, dtype=torch.float32)
    s = F.conv2d(mask.float(), ones, None, stride, padding, dilation)
    update = s.clamp(0, 1)
    ratio = winsize / (s + eps) * update
    return ratio, update


class _RenormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, raw, bias, mask, geom):
        kh, kw, sh, sw, ph, pw, dh, dw, winsize, eps = geom
        out, ratio, update = _ext.ext().partial_conv_renorm(
            raw, mask, bias, kh, kw, sh, sw, ph, pw, dh, dw, winsize, eps)
        ctx.save_for_backward(ratio, update)
        ctx.has_bias = bias is not None
        ctx.mark_non_differentiable(update)
        return out, update

    @staticmethod
    def backward(ctx, dout, _dupdate):
        ratio, update = ctx.saved_tensors
        draw = dout * (ratio * update).to(dout.dtype)
        dbias = (dout.float() * update).sum((0, 2, 3)) if ctx.has_bias else None
        return draw, dbias, None, None


def partial_conv_renorm(raw, mask, bias, kernel_size, stride, padding, dilation, winsize,
                        eps=1e-6):
    """Returns (out, update_mask) — update_mask has 1 channel (broadcastable)."""
    kh, kw = _pair(kernel_size)
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    dh, dw = _pair(dilation)
    if _ext.use_native(raw):
        mask = mask.to(raw.dtype) if mask.dtype not in (torch.float32, raw.dtype) else mask
        out, update = _RenormFn.apply(raw, bias, mask.detach(),
                                      (kh, kw, sh, sw, ph, pw, dh, dw, float(winsize), float(eps)))
        return out, update.to(raw.dtype)
    with torch.no_grad():
        ratio, update = _mask_stats_reference(mask.detach(), (kh, kw), (sh, sw), (ph, pw),
                                              (dh, dw), winsize, eps)
    out = raw * ratio.to(raw.dtype)
    if bias is not None:
        out = out + bias.reshape(1, -1, 1, 1).to(raw.dtype)
    out = out * update.to(raw.dtype)
    return out, update.to(raw.dtype)
