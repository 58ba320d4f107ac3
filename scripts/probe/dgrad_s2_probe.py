"""Stride-2 data gradient on k10 (phase decomposition) vs PyTorch fp32 and vs MIOpen: per-phase
errors on odd sizes, then timings on the SPADE discriminator / style-encoder shapes."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402


def check(B, cin, cout, H, W, k, s, p):
    torch.manual_seed(0)
    x = torch.randn(B, cin, H, W, device='cuda').to(torch.bfloat16)
    w = (torch.randn(cout, cin, k, k, device='cuda') / (cin * k * k) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    y = F.conv2d(x.float(), w.float(), None, s, p)
    dy = torch.randn_like(y).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ref = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), s, p)
    got = _ext.ext().conv2d_dgrad_strided_mfma(dy, w, H, W, s, p, p).float()
    torch.cuda.synchronize()
    errs = []
    for ry in range(s):
        for rx in range(s):
            e = (got[:, :, ry::s, rx::s] - ref[:, :, ry::s, rx::s]).abs().max().item()
            errs.append('(%d,%d) %.2e' % (ry, rx, e))
    print('check B%d %d->%d %dx%d k%d s%d p%d | ref max %.2f | %s' % (
        B, cin, cout, H, W, k, s, p, ref.abs().max().item(), '  '.join(errs)), flush=True)


def bench(B, cin, cout, H, W, k, s, p, reps=20):
    x = torch.randn(B, cin, H, W, device='cuda').to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, k, k, device='cuda') * 0.02).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(B, cout, Ho, Wo, device='cuda').to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)

    def k10():
        return _ext.ext().conv2d_dgrad_strided_mfma(dy, w, H, W, s, p, p)

    def miopen():
        return torch.ops.aten.convolution_backward(dy, x, w, None, (s, s), (p, p), (1, 1), False,
                                                   [0, 0], 1, [True, False, False])[0]
    out = {}
    for name, fn in (('k10s', k10), ('miopen', miopen)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        out[name] = e0.elapsed_time(e1) / reps
    fl = 2.0 * B * Ho * Wo * cout * cin * k * k
    print('bench %-34s k10s %.3f ms (%4.0f TF/s)  miopen %.3f ms (%4.0f TF/s)  %.2fx' % (
        '[%d,%d,%d,%d] k%d s%d' % (B, cin, H, W, k, s), out['k10s'],
        fl / out['k10s'] / 1e9, out['miopen'], fl / out['miopen'] / 1e9,
        out['miopen'] / out['k10s']), flush=True)


if __name__ == '__main__':
    for c in [(2, 64, 128, 15, 17, 3, 2, 1), (2, 64, 128, 16, 16, 3, 2, 1), (1, 64, 128, 15, 17, 3, 2, 1),
              (2, 64, 128, 15, 17, 4, 2, 1), (1, 64, 128, 11, 13, 5, 2, 2), (2, 128, 64, 9, 14, 1, 2, 0)]:
        check(*c)
    for c in [(4, 128, 128, 256, 512, 4, 2, 1), (8, 256, 128, 128, 256, 4, 2, 1),
              (8, 512, 256, 64, 128, 4, 2, 1), (4, 512, 512, 16, 32, 4, 2, 1),
              (8, 512, 512, 16, 32, 4, 2, 1), (8, 1024, 1024, 16, 32, 3, 2, 1),
              (4, 256, 128, 128, 256, 3, 2, 1), (4, 512, 256, 64, 128, 3, 2, 1)]:
        bench(*c)
