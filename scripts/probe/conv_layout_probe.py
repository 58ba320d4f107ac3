"""Probe MIOpen conv throughput for the SPADE 256x512 hot shapes: NCHW vs NHWC, bf16.

Run on the GPU box; prints one line per shape with fwd / fwd+bwd ms and TFLOP/s.
"""
import time, sys, os
import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True
dev = 'cuda'
B = 4
# (name, cin, cout, k, H, W, stride)
shapes = [
    ('head 3x3 2048->2048 16x32', 2048, 2048, 3, 16, 32, 1),
    ('up0 3x3 1024->1024 32x64', 1024, 1024, 3, 32, 64, 1),
    ('up1 3x3 512->512 64x128', 512, 512, 3, 64, 128, 1),
    ('up2 3x3 512->512 128x256', 512, 512, 3, 128, 256, 1),
    ('up2 3x3 256->256 128x256', 256, 256, 3, 128, 256, 1),
    ('spade mlp 5x5 185->128 128x256', 185, 128, 5, 128, 256, 1),
    ('spade gb 5x5 128->1024 128x256', 128, 1024, 5, 128, 256, 1),
    ('spade gb 5x5 128->2048 64x128', 128, 2048, 5, 64, 128, 1),
    ('D l0 4x4s2 188->128 256x512', 188, 128, 4, 256, 512, 2),
    ('D l1 4x4s2 128->256 128x256', 128, 256, 4, 128, 256, 2),
    ('vgg 3x3 64->64 256x512', 64, 64, 3, 256, 512, 1),
    ('vgg 3x3 128->128 128x256', 128, 128, 3, 128, 256, 1),
]

def bench(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3

for name, cin, cout, k, H, W, s in shapes:
    pad = (k - 1) // 2 if s == 1 else 1
    for fmt in ('nchw', 'nhwc'):
        x = torch.randn(B, cin, H, W, device=dev, dtype=torch.bfloat16)
        w = torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16) * 0.02
        if fmt == 'nhwc':
            x = x.contiguous(memory_format=torch.channels_last)
            w = w.contiguous(memory_format=torch.channels_last)
        x.requires_grad_(True); w.requires_grad_(True)
        y = F.conv2d(x, w, None, s, pad)
        Ho, Wo = y.shape[2], y.shape[3]
        flops = 2.0 * B * Ho * Wo * cout * cin * k * k
        g = torch.randn_like(y)
        tf = bench(lambda: F.conv2d(x, w, None, s, pad))
        def fb():
            yy = F.conv2d(x, w, None, s, pad)
            torch.autograd.grad(yy, (x, w), g)
        tfb = bench(fb)
        print(f'{name:34s} {fmt} fwd {tf:7.3f} ms {flops/tf/1e9:7.1f} TF/s | fwd+bwd {tfb:7.3f} ms {3*flops/tfb/1e9:7.1f} TF/s', flush=True)
