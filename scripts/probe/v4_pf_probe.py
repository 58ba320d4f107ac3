"""k10 v4 with vs without the cross-barrier fragment prefetch (IMAGINAIRE_AMD_V4_PF 1 / 0) on the
SPADE-step stride-1 shapes, interleaved in one process (cdna guide rule 24).

    python scripts/probe/v4_pf_probe.py
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
    # name, B, cin, cout, k, H, W, pad
    ('G head 3x3 2048->2048 16x32', 4, 2048, 2048, 3, 16, 32, 1),
    ('G up0 3x3 1024->1024 32x64', 4, 1024, 1024, 3, 32, 64, 1),
    ('G up1 3x3 512->512 64x128', 4, 512, 512, 3, 64, 128, 1),
    ('G up2 3x3 512->512 128x256', 4, 512, 512, 3, 128, 256, 1),
    ('G up3 3x3 256->128 256x512', 4, 256, 128, 3, 256, 512, 1),
    ('spade mlp 5x5 192->128 256x512', 4, 192, 128, 5, 256, 512, 2),
    ('spade gb 5x5 128->1024 128x256', 4, 128, 1024, 5, 128, 256, 2),
    ('spade gb 5x5 128->512 256x512', 4, 128, 512, 5, 256, 512, 2),
    ('spade gb 5x5 128->2048 64x128', 4, 128, 2048, 5, 64, 128, 2),
    ('spade gb 5x5 128->4096 16x32', 4, 128, 4096, 5, 16, 32, 2),
    ('dgrad-as-conv 5x5 1024->128 128x256', 4, 1024, 128, 5, 128, 256, 2),
    ('dgrad-as-conv 3x3 512->256 128x256', 4, 512, 256, 3, 128, 256, 1),
    ('vgg 3x3 256->256 64x128', 4, 256, 256, 3, 64, 128, 1),
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
os.environ['IMAGINAIRE_AMD_CONV_V'] = '4'
torch.manual_seed(0)
tot = {'0': 0.0, '1': 0.0}
for name, B, cin, cout, k, H, W, pad in shapes:
    x = torch.randn(B, cin, H, W, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(cout, cin, k, k, device='cuda', dtype=torch.bfloat16) * 0.02).contiguous(
        memory_format=CL)
    bias = torch.randn(cout, device='cuda', dtype=torch.float32)
    ref = F.leaky_relu(F.conv2d(x.float(), w.float(), bias, 1, pad), 0.2)
    flops = 2.0 * B * H * W * cout * cin * k * k
    errs, ts = {}, {'0': [], '1': []}
    for v in ('0', '1'):
        os.environ['IMAGINAIRE_AMD_V4_PF'] = v
        y = ext.conv2d_mfma(x, w, bias, 1, 1, pad, pad, 1, 1, 0.2)
        errs[v] = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    for rnd in range(3):
        for v in ('0', '1'):
            os.environ['IMAGINAIRE_AMD_V4_PF'] = v
            ts[v].append(timeit(lambda: ext.conv2d_mfma(x, w, bias, 1, 1, pad, pad, 1, 1, 0.2)))
    t0, t1 = min(ts['0']), min(ts['1'])
    tot['0'] += t0
    tot['1'] += t1
    print('%-38s | pf0 %7.3f ms %6.0f TF/s err %.1e | pf1 %7.3f ms %6.0f TF/s err %.1e | %.3fx'
          % (name, t0, flops / t0 / 1e9, errs['0'], t1, flops / t1 / 1e9, errs['1'], t0 / t1),
          flush=True)
    for v in ('0', '1'):
        assert errs[v] < 2e-2, (name, v, errs[v])
print('sum over shapes: pf0 %.3f ms, pf1 %.3f ms (%.3fx)' % (tot['0'], tot['1'], tot['0'] / tot['1']))
