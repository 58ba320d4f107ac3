"""Does zero-padding an odd input-channel count help MIOpen's NHWC bf16 kernels?

    python scripts/probe/conv_pad_probe.py

For each SPADE-step conv whose Cin is not a multiple of 32 (label maps:
183 classes + don't-care + edge = 185; D input label+image = 188), time
fwd+bwd at the native Cin and at Cin rounded up to 192 (zero channels),
including the cost of materialising the padded activation.
"""
import time

import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True
dev = 'cuda'
B = 4
CL = torch.channels_last
shapes = [
    # name, cin, cout, k, H, W, stride, input needs grad
    ('spade mlp 5x5 185->128 256x512', 185, 128, 5, 256, 512, 1, False),
    ('spade mlp 5x5 185->128 128x256', 185, 128, 5, 128, 256, 1, False),
    ('spade mlp 5x5 185->128 64x128', 185, 128, 5, 64, 128, 1, False),
    ('D l0 4x4s2 188->128 256x512', 188, 128, 4, 256, 512, 2, True),
    ('D l0 4x4s2 188->128 128x256', 188, 128, 4, 128, 256, 2, True),
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


for name, cin, cout, k, H, W, s, xgrad in shapes:
    pad = (k - 1) // 2 if s == 1 else 1
    x = torch.randn(B, cin, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16) * 0.02).contiguous(
        memory_format=CL).requires_grad_(True)
    x.requires_grad_(xgrad)
    y = F.conv2d(x.detach(), w.detach(), None, s, pad)
    g = torch.randn_like(y)
    ins = (x, w) if xgrad else (w,)

    def native():
        yy = F.conv2d(x, w, None, s, pad)
        torch.autograd.grad(yy, ins, g)

    cp = (cin + 31) // 32 * 32

    def padded():
        xp = F.pad(x, (0, 0, 0, 0, 0, cp - cin)).contiguous(memory_format=CL)
        wp = F.pad(w, (0, 0, 0, 0, 0, cp - cin)).contiguous(memory_format=CL)
        yy = F.conv2d(xp, wp, None, s, pad)
        torch.autograd.grad(yy, ins, g)

    xp0 = F.pad(x.detach(), (0, 0, 0, 0, 0, cp - cin)).contiguous(memory_format=CL)
    wp0 = F.pad(w.detach(), (0, 0, 0, 0, 0, cp - cin)).contiguous(memory_format=CL).requires_grad_(True)
    xp0.requires_grad_(xgrad)
    ins0 = (xp0, wp0) if xgrad else (wp0,)

    def prepadded():
        yy = F.conv2d(xp0, wp0, None, s, pad)
        torch.autograd.grad(yy, ins0, g)

    flops = (3 if xgrad else 2) * 2.0 * B * y.shape[2] * y.shape[3] * cout * cin * k * k
    for tag, fn in (('native', native), ('pad%d' % cp, padded), ('prepad%d' % cp, prepadded)):
        ms = bench(fn)
        print('%-34s %-9s fwd+bwd %8.3f ms %7.1f TF/s(useful)' % (name, tag, ms, flops / ms / 1e9),
              flush=True)
