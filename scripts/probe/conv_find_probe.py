"""MIOpen find cost vs steady-state speed for SPADE-step conv shapes (NHWC bf16).

    python scripts/probe/conv_find_probe.py [bench|nobench]

Prints, per shape: first fwd+bwd call latency (includes MIOpen find/compile)
and steady-state fwd+bwd ms / TFLOP/s.
"""
import sys
import time

import torch
import torch.nn.functional as F

mode = sys.argv[1] if len(sys.argv) > 1 else 'bench'
torch.backends.cudnn.benchmark = mode == 'bench'
dev = 'cuda'
B = 4
shapes = [
    ('up1 3x3 512->512 64x128', 512, 512, 3, 64, 128, 1),
    ('up2 3x3 256->256 128x256', 256, 256, 3, 128, 256, 1),
    ('spade mlp 5x5 185->128 128x256', 185, 128, 5, 128, 256, 1),
    ('spade gb 5x5 128->1024 128x256', 128, 1024, 5, 128, 256, 1),
    ('D l0 4x4s2 188->128 256x512', 188, 128, 4, 256, 512, 2),
    ('vgg 3x3 64->64 256x512', 64, 64, 3, 256, 512, 1),
    ('enc 3x3s2 3->64 256x512', 3, 64, 3, 256, 512, 2),
    ('img 3x3 64->3 256x512', 64, 3, 3, 256, 512, 1),
]


def run(x, w, s, pad, g):
    y = F.conv2d(x, w, None, s, pad)
    torch.autograd.grad(y, (x, w), g)


for name, cin, cout, k, H, W, s in shapes:
    pad = (k - 1) // 2 if s == 1 else 1
    x = torch.randn(B, cin, H, W, device=dev, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    w = (torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16) * 0.02).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    y = F.conv2d(x.detach(), w.detach(), None, s, pad)
    g = torch.randn_like(y)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(x, w, s, pad, g)
    torch.cuda.synchronize()
    first = time.perf_counter() - t0
    for _ in range(3):
        run(x, w, s, pad, g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        run(x, w, s, pad, g)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 10 * 1e3
    flops = 3 * 2.0 * B * y.shape[2] * y.shape[3] * cout * cin * k * k
    print('%-32s %s first %8.2f s | fwd+bwd %8.3f ms %7.1f TF/s' % (
        name, mode, first, ms, flops / ms / 1e9), flush=True)
