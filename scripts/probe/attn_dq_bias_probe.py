"""Systematic error of the k16 attention backward: queries sharing a common offset (a 1x1 conv
bias, as in NonLocal2dBlock's theta) make the per-channel SUM of dq over all queries — the bias
gradient — sensitive to any biased rounding in dq. Compares k16, PyTorch SDPA under bf16 and the
fp32 formulation on the same bf16-rounded inputs.

    python scripts/probe/attn_dq_bias_probe.py
"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from imaginaire_amd.ops import attention as A  # noqa: E402


def run(B, Lq, Lk, d, dv, qoff, kscale):
    torch.manual_seed(0)
    q = (torch.randn(B, Lq, d, device='cuda') + qoff * torch.randn(d, device='cuda')).to(
        torch.bfloat16)
    k = (kscale * torch.randn(B, Lk, d, device='cuda')).to(torch.bfloat16)
    v = torch.randn(B, Lk, dv, device='cuda').to(torch.bfloat16)
    go = torch.randn(B, Lq, dv, device='cuda')
    res = {}
    for tag in ('k16', 'sdpa16', 'fp32'):
        qi, ki, vi = (t.clone().float().requires_grad_(True) if tag == 'fp32' else
                      t.clone().requires_grad_(True) for t in (q, k, v))
        if tag == 'k16':
            o = A.fused_attention(qi, ki, vi, 1.0)
        elif tag == 'sdpa16':
            o = F.scaled_dot_product_attention(qi[:, None], ki[:, None], vi[:, None],
                                               scale=1.0)[:, 0]
        else:
            o = A.attention_reference(qi, ki, vi, 1.0)
        o.backward(go.to(o.dtype))
        res[tag] = (o.detach().float(), qi.grad.float(), ki.grad.float(), vi.grad.float())
    r = res['fp32']
    for tag in ('k16', 'sdpa16'):
        a = res[tag]
        msg = []
        for name, x, y in zip(('o', 'dq', 'dk', 'dv'), a, r):
            rel = float((x - y).norm() / y.norm())
            cs_x, cs_y = x.sum((0, 1)), y.sum((0, 1))
            crel = float((cs_x - cs_y).norm() / cs_y.norm())
            mean_off = float((cs_x - cs_y).mean() / cs_y.abs().mean())
            msg.append('%s rel %.2e colsum rel %.2e (mean offset %.2e)' % (name, rel, crel,
                                                                        mean_off))
        print('B%d Lq%d Lk%d d%d dv%d qoff %.1f ks %.1f %-6s: %s' % (
            B, Lq, Lk, d, dv, qoff, kscale, tag, ' | '.join(msg)), flush=True)


if __name__ == '__main__':
    torch.cuda.set_device(0)
    for args in ((2, 1024, 256, 32, 128, 0.0, 1.0), (2, 1024, 256, 32, 128, 3.0, 1.0),
                 (2, 1024, 256, 32, 128, 3.0, 0.3), (2, 1024, 256, 64, 256, 2.0, 0.5),
                 (1, 4096, 1024, 32, 128, 3.0, 0.5)):
        run(*args)
