"""Check the k16 attention backward on the operands the few-shot vid2vid model actually feeds
it: every ``_FusedAttentionFn.backward`` of one HIP-bf16 training iteration (unit config, K = 2)
also computes dq / dk / dv with the explicit fp32 formulation (bmm -> softmax -> bmm) from the
same saved bf16 q, k, v and incoming gradient, and prints relative errors and cosines, plus the
energy range (the unscaled few-shot softmax is sharply peaked).

    python scripts/probe/fs_attn_dq_probe.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

from imaginaire_amd.ops import attention as A  # noqa: E402

_orig = A._FusedAttentionFn.backward


def _checked(ctx, do):
    dq, dk, dv, none = _orig(ctx, do)
    q, k, v, o, lse = ctx.saved_tensors
    with torch.enable_grad():
        qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
        s = torch.bmm(qr, kr.transpose(1, 2)) * ctx.scale
        ref = torch.bmm(torch.softmax(s, dim=2), vr)
        gq, gk, gv = torch.autograd.grad(ref, (qr, kr, vr), do.float())

    def stats(a, b):
        a = a.float().reshape(-1)
        b = b.reshape(-1)
        rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
        cos = float(torch.dot(a, b) / (a.norm() * b.norm()).clamp_min(1e-30))
        return 'rel %.3g cos %.4f |ref| %.3g' % (rel, cos, float(b.norm()))
    p = torch.softmax(s.detach(), dim=2)
    print('[attn-bwd] q %s k %s v %s scale %.3g | energy min %.1f max %.1f, max p %.3f' % (
        tuple(q.shape), tuple(k.shape), tuple(v.shape), ctx.scale, float(s.min()),
        float(s.max()), float(p.max(dim=2).values.mean())), flush=True)
    print('[attn-bwd]   dq %s' % stats(dq, gq), flush=True)
    print('[attn-bwd]   dk %s' % stats(dk, gk), flush=True)
    print('[attn-bwd]   dv %s' % stats(dv, gv), flush=True)
    o_ref = ref.detach()
    print('[attn-bwd]   o  %s' % stats(o, o_ref), flush=True)
    return dq, dk, dv, none


A._FusedAttentionFn.backward = staticmethod(_checked)

import test_model_parity_gpu as P  # noqa: E402
import tempfile  # noqa: E402

torch.cuda.set_device(0)
P._iteration('fs_vid2vid_face.yaml', 'O1', False, tempfile.mkdtemp(), seq_len=2,
             overrides=[('data.initial_few_shot_K', 2)])
print('done', flush=True)
