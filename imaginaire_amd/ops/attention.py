"""Fused attention ``softmax(scale * q k^T) v`` over a long key axis (k16, ``csrc/attention.hip``).

The few-shot vid2vid reference-frame attention (reference generators/fs_vid2vid.py:944-951)
materialises a B x (K*HW) x HW energy matrix, softmaxes it over the reference positions and
multiplies it into the features with a second bmm. Here one HIP kernel streams the keys through
LDS with an online softmax (MFMA 16x16x32 bf16, fp32 statistics) and writes only the output and
a per-query log-sum-exp; the backward recomputes the probabilities from it in two kernels (dK/dV
per key block, dQ per query block; deterministic, no atomics).

``fused_attention(q, k, v, scale)`` takes q [B, Lq, d], k [B, Lk, d], v [B, Lk, dv] of any float
dtype and returns [B, Lq, dv] in the caller's compute dtype (autocast's, else q's; the kernel
itself computes in bf16). Head dims are zero-padded to the kernel's
sizes (d -> 32 / 64 / 128, dv -> a multiple of 32): zero columns change no dot product; value
widths above 288 run as column chunks (the few-shot vid2vid recipe's 128 + 128 + K channels
fit one 288-wide pass).
Shapes the kernel does not take (sequence lengths not multiples of 64, d > 128) and CPU tensors
run PyTorch's ``scaled_dot_product_attention``.

    IMAGINAIRE_AMD_FUSED_ATTN_KERNEL=0   PyTorch SDPA everywhere (A/B switch)
"""
import os

import torch
import torch.nn.functional as F

from imaginaire_amd.ops import _ext

_NATIVE = os.environ.get('IMAGINAIRE_AMD_FUSED_ATTN_KERNEL', '1') != '0'


def _pad_head(d):
    for c in (32, 64, 128):
        if d <= c:
            return c
    return None


def _pad_value(dv):
    c = (dv + 31) // 32 * 32
    if c == 224:
        c = 256
    return c if c <= 288 else None


def native_ok(q, k, v):
    return (_NATIVE and q.is_cuda and _ext.use_native(q) and q.dim() == 3 and
            q.shape[1] % 64 == 0 and k.shape[1] % 64 == 0 and _pad_head(q.shape[2]) is not None)


def _value_chunks(dv):
    """Column chunks of a value width the kernel takes: one chunk up to 288 (the few-shot
    recipe's 258), else full 256-wide chunks, then the remainder. Softmax(q k^T) is the same for every chunk and the backward is linear in the
    chunks' dP (dS = P * (dP - rowsum(dO * O)) sums over them), so chunk outputs concatenate and
    chunk gradients of q and k add up."""
    if dv <= 288:
        return [(0, dv)]
    out, c0 = [], 0
    while c0 < dv:
        w = min(256, dv - c0)
        out.append((c0, w))
        c0 += w
    return out


class _FusedAttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale):
        o, lse = _ext.ext().attention_fwd(q, k, v, float(scale))
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.scale = float(scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = _ext.ext().attention_bwd(q, k, v, o, lse, do.contiguous(), ctx.scale)
        return dq, dk, dv, None


def attention_reference(q, k, v, scale=1.0):
    """The reference formulation in the input dtype: explicit scores, softmax over keys, bmm."""
    a = torch.softmax(torch.bmm(q, k.transpose(1, 2)) * scale, dim=2)
    return torch.bmm(a, v)


def fused_attention(q, k, v, scale=1.0):
    if not native_ok(q, k, v):
        dt = q.dtype
        with torch.autocast(q.device.type, enabled=False):
            return F.scaled_dot_product_attention(q.unsqueeze(1), k.to(dt).unsqueeze(1),
                                                  v.to(dt).unsqueeze(1), scale=scale).squeeze(1)
    # the kernel computes in bf16; the result comes back in the compute dtype of the caller
    # (autocast's, else q's), so an fp32 caller never receives a bf16 tensor
    out_dt = torch.get_autocast_dtype('cuda') if torch.is_autocast_enabled('cuda') else q.dtype
    d, dv = q.shape[2], v.shape[2]
    D = _pad_head(d)
    with torch.autocast('cuda', enabled=False):
        qp = F.pad(q.to(torch.bfloat16), (0, D - d)).contiguous()
        kp = F.pad(k.to(torch.bfloat16), (0, D - d)).contiguous()
        vb = v.to(torch.bfloat16)
        outs = []
        for c0, w in _value_chunks(dv):
            DV = _pad_value(w)
            vp = F.pad(vb[:, :, c0:c0 + w], (0, DV - w)).contiguous()
            o = _FusedAttentionFn.apply(qp, kp, vp, scale)
            outs.append(o[:, :, :w] if DV != w else o)
    o = outs[0] if len(outs) == 1 else torch.cat(outs, 2)
    return o if o.dtype == out_dt else o.to(out_dt)
