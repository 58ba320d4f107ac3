"""Few-shot vid2vid reference pooling (reference generators/fs_vid2vid.py:780-788):
``prod[b, c, c'] = sum_p conv[b, c, p] * softmax_c'(label)[b, c', p]``.

The reference writes it as ``softmax(dim=1)`` + ``torch.bmm``. On channels-last activations
PyTorch runs that softmax as a strided "spatial" softmax and the bmm through hipBLASLt with
a transposed operand. Here:

* the softmax over channels is the k15 kernel (``csrc/channel_softmax.hip``: one contiguous
  row per pixel, group-of-lanes reductions, one read + one write), forward and backward;
* the pooled product is a per-sample 1x1 weight-gradient GEMM — K = pixels, a tiny c x c'
  output — on the batched k11 MFMA kernel (one launch, grid z = sample), and its backward two
  per-sample 1x1 k10 convolutions (d conv = dprod . s, d s = dprod^T . conv).

CPU / unsupported inputs run the reference formulation.
"""
import os

import torch

from imaginaire_amd.ops import _ext

# IMAGINAIRE_AMD_FEW_SHOT_POOL=0: the reference formulation (softmax + bmm) everywhere
_NATIVE_POOL = os.environ.get('IMAGINAIRE_AMD_FEW_SHOT_POOL', '1') == '1'

_CL = torch.channels_last


def _round64(c):
    return (c + 63) // 64 * 64


def _csm_native(x):
    c = x.shape[1] if x.dim() == 4 else 0
    return (x.dim() == 4 and x.is_cuda and x.dtype == torch.bfloat16 and _ext.use_native(x) and
            16 <= c <= 4096 and (c & (c - 1)) == 0)


class _ChannelSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = _ext.ext().channel_softmax_fwd(x.contiguous(memory_format=_CL))
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, = ctx.saved_tensors
        return _ext.ext().channel_softmax_bwd(y, dy.to(torch.bfloat16).contiguous(memory_format=_CL))


def channel_softmax(x):
    """``torch.softmax(x, dim=1)`` of a 4-D activation (bf16 channels-last on the k15 kernel)."""
    if _csm_native(x):
        return _ChannelSoftmax.apply(x)
    return torch.softmax(x, dim=1)


def _pad_c(t, c):
    from imaginaire_amd.ops.conv import _pad_channels
    return _pad_channels(t, c, torch.bfloat16)


class _SoftmaxPool(torch.autograd.Function):
    """prod[b, c, c'] = sum_p a[b, c, p] * s[b, c', p] (a, s: [B, C, H, W] bf16)."""

    @staticmethod
    def forward(ctx, a, s):
        B, c, H, W = a.shape
        c2 = s.shape[1]
        ca, cs = _round64(c), _round64(c2)
        ap, sp = _pad_c(a, ca), _pad_c(s, cs)
        # k11 per-sample 1x1 weight gradient: g[b * ca + i, j] = sum_p ap[b, i, p] * sp[b, j, p]
        g = _ext.ext().conv2d_wgrad_mfma(ap, sp, 1, 1, 1, 1, 0, 0, 1, 1, -1, -1, False, B)
        prod = g.reshape(B, ca, cs)[:, :c, :c2]
        ctx.save_for_backward(ap, sp)
        ctx.conf = (c, c2, a.dtype, s.dtype)
        return prod.to(torch.bfloat16)

    @staticmethod
    def backward(ctx, dprod):
        ap, sp = ctx.saved_tensors
        c, c2, adt, sdt = ctx.conf
        B, ca = ap.shape[0], ap.shape[1]
        cs = sp.shape[1]
        X = _ext.ext()
        dp = torch.zeros((B, ca, cs), dtype=torch.bfloat16, device=dprod.device)
        dp[:, :c, :c2] = dprod
        da = ds = None
        if ctx.needs_input_grad[0]:
            # da[b, i, p] = sum_j dp[b, i, j] sp[b, j, p]: 1x1 conv of sp with weight dp[b]
            w1 = dp.reshape(B * ca, cs, 1, 1).contiguous(memory_format=_CL)
            da = X.conv2d_mfma(sp, w1, None, 1, 1, 0, 0, 1, 1, 1.0, B)[:, :c].to(adt)
        if ctx.needs_input_grad[1]:
            # ds[b, j, p] = sum_i dp[b, i, j] ap[b, i, p]: 1x1 conv of ap with weight dp[b]^T
            w2 = dp.transpose(1, 2).reshape(B * cs, ca, 1, 1).contiguous(memory_format=_CL)
            ds = X.conv2d_mfma(ap, w2, None, 1, 1, 0, 0, 1, 1, 1.0, B)[:, :c2].to(sdt)
        return da, ds


def _pool_native(a, s):
    if not (_NATIVE_POOL and a.is_cuda and a.dim() == 4 and s.dim() == 4 and _ext.use_native(a) and
            a.shape[0] == s.shape[0] and a.shape[2:] == s.shape[2:]):
        return False
    dt = torch.get_autocast_dtype('cuda') if torch.is_autocast_enabled('cuda') else a.dtype
    if dt != torch.bfloat16:
        return False
    B, _, H, W = a.shape
    # k11 / k10 32-bit buffer offsets and per-sample pixel rows
    return H * W >= 64 and max(_round64(a.shape[1]), _round64(s.shape[1])) * B * H * W * 2 < (1 << 30)


def softmax_pool(conv, label):
    """``bmm(conv.reshape(b, c, hw), softmax(label, 1).reshape(b, c', hw).transpose(1, 2))``
    -> [b, c, c'] (reference generators/fs_vid2vid.py:780-788)."""
    b, c, h, w = conv.shape
    if _pool_native(conv, label):
        with torch.autocast('cuda', enabled=False):
            a = conv.to(torch.bfloat16).contiguous(memory_format=_CL)
            s = channel_softmax(label.to(torch.bfloat16).contiguous(memory_format=_CL))
            if not _csm_native(s):
                s = s.contiguous(memory_format=_CL)
            return _SoftmaxPool.apply(a, s)
    sm = torch.softmax(label, dim=1)
    return torch.bmm(conv.reshape(b, c, h * w), sm.reshape(b, label.shape[1], h * w).transpose(1, 2))
