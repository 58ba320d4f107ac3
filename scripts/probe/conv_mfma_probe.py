"""k10 MFMA implicit-GEMM conv vs MIOpen on the SPADE-step conv shapes (NHWC bf16).

    python scripts/probe/conv_mfma_probe.py

Per shape: forward-only and forward+backward (dx, dW) time for MIOpen (packed NHWC,
odd channels zero-padded to a multiple of 32) and for the k10 path (MFMA forward and
stride-1 dgrad, MIOpen wgrad), plus a max-abs-error check of the k10 forward.
"""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import conv as C  # noqa: E402

torch.backends.cudnn.benchmark = False
dev = 'cuda'
CL = torch.channels_last
C._MFMA_MIN_BLOCKS = 0
shapes = [
    # name, B, cin, cout, k, H, W, stride, x needs grad
    ('G head 3x3 2048->2048 16x32', 4, 2048, 2048, 3, 16, 32, 1, True),
    ('G up0 3x3 1024->1024 32x64', 4, 1024, 1024, 3, 32, 64, 1, True),
    ('G up1 3x3 512->512 64x128', 4, 512, 512, 3, 64, 128, 1, True),
    ('G up2 3x3 256->256 128x256', 4, 256, 256, 3, 128, 256, 1, True),
    ('G up3 3x3 128->128 256x512', 4, 128, 128, 3, 256, 512, 1, True),
    ('spade mlp 5x5 185->128 256x512', 4, 185, 128, 5, 256, 512, 1, False),
    ('spade mlp 5x5 185->128 64x128', 4, 185, 128, 5, 64, 128, 1, False),
    ('spade gb 5x5 128->256 256x512', 4, 128, 256, 5, 256, 512, 1, True),
    ('spade gb 5x5 128->512 128x256', 4, 128, 512, 5, 128, 256, 1, True),
    ('spade gb 5x5 128->2048 32x64', 4, 128, 2048, 5, 32, 64, 1, True),
    ('spade gb 5x5 128->4096 16x32', 4, 128, 4096, 5, 16, 32, 1, True),
    ('D l0 4x4s2 188->128 256x512', 4, 188, 128, 4, 256, 512, 2, True),
    ('D l1 4x4s2 128->256 128x256', 4, 128, 256, 4, 128, 256, 2, True),
    ('D l2 4x4s2 256->512 64x128', 4, 256, 512, 4, 64, 128, 2, True),
    ('vgg 3x3 64->64 256x512', 4, 64, 64, 3, 256, 512, 1, True),
    ('vgg 3x3 128->128 128x256', 4, 128, 128, 3, 128, 256, 1, True),
    ('vgg 3x3 256->256 64x128', 4, 256, 256, 3, 64, 128, 1, True),
]


def bench(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


for name, B, cin, cout, k, H, W, s, xg in shapes:
    pad = (k - 1) // 2 if s == 1 else 1
    x = torch.randn(B, cin, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16) * 0.02).contiguous(
        memory_format=CL)
    x.requires_grad_(xg)
    w.requires_grad_(True)
    ins = (x, w) if xg else (w,)
    with torch.no_grad():
        y_ref = F.conv2d(x.float(), w.float(), None, s, pad)
    g = torch.randn_like(y_ref).to(torch.bfloat16).contiguous(memory_format=CL)
    flops_f = 2.0 * B * y_ref.shape[2] * y_ref.shape[3] * cout * cin * k * k
    flops_fb = flops_f * (3 if xg else 2)
    res = {}
    for tag, on in (('miopen', '0'), ('mfma', '1')):

        os.environ['IMAGINAIRE_AMD_MFMA_CONV'] = on

        def fwd():
            with torch.no_grad():
                return C.conv2d(x, w, None, s, pad)

        def fb():
            yy = C.conv2d(x, w, None, s, pad)
            torch.autograd.grad(yy, ins, g)

        y = fwd()
        err = (y.float() - y_ref).abs().max().item() / max(1e-6, y_ref.abs().max().item())
        tf = bench(fwd)
        tfb = bench(fb)
        res[tag] = (tf, tfb, err)
    print('%-32s fwd miopen %7.3f ms %6.0f TF/s | mfma %7.3f ms %6.0f TF/s (relerr %.1e) || '
          'fwd+bwd miopen %7.3f | k10 %7.3f ms' % (
              name, res['miopen'][0], flops_f / res['miopen'][0] / 1e9, res['mfma'][0],
              flops_f / res['mfma'][0] / 1e9, res['mfma'][2], res['miopen'][1], res['mfma'][1]),
          flush=True)

print('--- weight gradient: MIOpen wrw vs k11 ---', flush=True)
ext = C._ext.ext()
for name, B, cin, cout, k, H, W, s, xg in shapes:
    pad = (k - 1) // 2 if s == 1 else 1
    cp = C._round_up(cin, 64)
    x = torch.randn(B, cp, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(cout, cp, k, k, device=dev, dtype=torch.bfloat16) * 0.02).contiguous(
        memory_format=CL)
    ho = (H + 2 * pad - k) // s + 1
    wo = (W + 2 * pad - k) // s + 1
    g = torch.randn(B, cout, ho, wo, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
    flops = 2.0 * B * ho * wo * cout * cp * k * k

    def miopen():
        return torch.ops.aten.convolution_backward(g, x, w, None, (s, s), (pad, pad), (1, 1),
                                                   False, [0, 0], 1, [False, True, False])[1]

    def k11():
        return ext.conv2d_wgrad_mfma(g, x, k, k, s, s, pad, pad, 1, 1)

    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, g.float(), s, pad)
    err = (k11().float() - ref).abs().max().item() / max(1e-6, ref.abs().max().item())
    tm, tk = bench(miopen), bench(k11)
    print('%-32s wgrad miopen %7.3f ms %6.0f TF/s | k11 %7.3f ms %6.0f TF/s (relerr %.1e)' % (
        name, tm, flops / tm / 1e9, tk, flops / tk / 1e9, err), flush=True)

print('--- k10 forward tile: BM=128 (4 waves, 2 blocks/CU) vs BM=256 (8 waves) ---', flush=True)
for name, B, cin, cout, k, H, W, s, xg in shapes:
    pad = (k - 1) // 2 if s == 1 else 1
    cp = C._round_up(cin, 64)
    x = torch.randn(B, cp, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(cout, cp, k, k, device=dev, dtype=torch.bfloat16) * 0.02).contiguous(
        memory_format=CL)
    ho = (H + 2 * pad - k) // s + 1
    wo = (W + 2 * pad - k) // s + 1
    flops = 2.0 * B * ho * wo * cout * cp * k * k
    res = []
    for bm in ('128', '256'):
        os.environ['IMAGINAIRE_AMD_CONV_BM'] = bm
        y = ext.conv2d_mfma(x, w, None, s, s, pad, pad, 1, 1, 1.0)
        t = bench(lambda: ext.conv2d_mfma(x, w, None, s, s, pad, pad, 1, 1, 1.0))
        res.append((t, y))
    os.environ.pop('IMAGINAIRE_AMD_CONV_BM')
    same = (res[0][1].float() - res[1][1].float()).abs().max().item()
    print('%-32s BM128 %7.3f ms %6.0f TF/s | BM256 %7.3f ms %6.0f TF/s | max diff %.1e' % (
        name, res[0][0], flops / res[0][0] / 1e9, res[1][0], flops / res[1][0] / 1e9, same),
        flush=True)
