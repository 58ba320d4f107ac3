"""k10 v1 (128x128, 2-stage, vmcnt(0) per step) vs v2 (256x128, 3-stage ring, counted vmcnt)
on the SPADE-step forward / dgrad conv shapes, interleaved in one process (cdna guide rule 24).

    python scripts/probe/conv_v2_probe.py
"""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402

CL = torch.channels_last
shapes = [
    # name, B, cin, cout, k, H, W, stride, pad
    ('G head 3x3 2048->2048 16x32', 4, 2048, 2048, 3, 16, 32, 1, 1),
    ('G up0 3x3 1024->1024 32x64', 4, 1024, 1024, 3, 32, 64, 1, 1),
    ('G up1 3x3 512->512 64x128', 4, 512, 512, 3, 64, 128, 1, 1),
    ('G up2 3x3 512->512 128x256', 4, 512, 512, 3, 128, 256, 1, 1),
    ('G up3 3x3 256->128 256x512', 4, 256, 128, 3, 256, 512, 1, 1),
    ('spade mlp 5x5 192->128 256x512', 4, 192, 128, 5, 256, 512, 1, 2),
    ('spade mlp 5x5 192->128 64x128', 4, 192, 128, 5, 64, 128, 1, 2),
    ('spade gb 5x5 128->1024 128x256', 4, 128, 1024, 5, 128, 256, 1, 2),
    ('spade gb 5x5 128->512 256x512', 4, 128, 512, 5, 256, 512, 1, 2),
    ('spade gb 5x5 128->2048 64x128', 4, 128, 2048, 5, 64, 128, 1, 2),
    ('spade gb 5x5 128->4096 16x32', 4, 128, 4096, 5, 16, 32, 1, 2),
    ('dgrad gb 5x5 1024->128 128x256', 4, 1024, 128, 5, 128, 256, 1, 2),
    ('dgrad gb 5x5 4096->128 32x64', 4, 4096, 128, 5, 32, 64, 1, 2),
    ('dgrad gb 5x5 2048->128 64x128', 4, 2048, 128, 5, 64, 128, 1, 2),
    ('dgrad gb 5x5 512->128 256x512', 4, 512, 128, 5, 256, 512, 1, 2),
    ('spade mlp 5x5 192->128 128x256', 4, 192, 128, 5, 128, 256, 1, 2),
    ('dgrad G 3x3 512->256 128x256', 4, 512, 256, 3, 128, 256, 1, 1),
    ('D l1 4x4s2 128->256 128x256', 4, 128, 256, 4, 128, 256, 2, 1),
    ('D l2 4x4s2 256->512 64x128', 4, 256, 512, 4, 64, 128, 2, 1),
    ('vgg 3x3 128->128 128x256', 4, 128, 128, 3, 128, 256, 1, 1),
    ('vgg 3x3 256->256 64x128', 4, 256, 256, 3, 64, 128, 1, 1),
]


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


ext = _ext.ext()
VERS = sys.argv[1].split(',') if len(sys.argv) > 1 else ['1', '2', '3']
torch.manual_seed(0)
for name, B, cin, cout, k, H, W, s, pad in shapes:
    x = torch.randn(B, cin, H, W, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(cout, cin, k, k, device='cuda', dtype=torch.bfloat16) * 0.02).contiguous(
        memory_format=CL)
    bias = torch.randn(cout, device='cuda', dtype=torch.float32)
    ref = F.leaky_relu(F.conv2d(x.float(), w.float(), bias, s, pad), 0.2)
    Ho, Wo = ref.shape[2], ref.shape[3]
    flops = 2.0 * B * Ho * Wo * cout * cin * k * k
    res = {}
    errs = {}
    vers = [v for v in VERS if not (v == '3' and cout % 256)]
    for v in vers:
        os.environ['IMAGINAIRE_AMD_CONV_V'] = v
        y = ext.conv2d_mfma(x, w, bias, s, s, pad, pad, 1, 1, 0.2)
        errs[v] = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    ts = {v: [] for v in vers}
    for rnd in range(3):
        for v in vers:
            os.environ['IMAGINAIRE_AMD_CONV_V'] = v
            ts[v].append(timeit(lambda: ext.conv2d_mfma(x, w, bias, s, s, pad, pad, 1, 1, 0.2)))
    line = '%-34s' % name
    for v in vers:
        t = min(ts[v])
        line += ' | v%s %7.3f ms %6.0f TF/s err %.1e' % (v, t, flops / t / 1e9, errs[v])
    for v in vers[1:]:
        line += ' | v%s/v1 %.2fx' % (v, min(ts['1']) / min(ts[v]))
    print(line, flush=True)
    for v in vers:
        assert errs[v] < 2e-2, (name, v, errs[v])
