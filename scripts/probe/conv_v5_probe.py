"""k10 v5 (256 x 256 tile, 8 waves of 128 x 64) vs v4 (256 x 128, 8 waves of 64 x 64) on the
SPADE-step conv shapes with >= 256 output channels, interleaved in one process (cdna guide
rule 24), random bf16 operands. dgrad rows are the stride-1 data gradients as k10 runs them
(a conv of dy with the flipped weight: N = Cin of the forward).

    python scripts/probe/conv_v5_probe.py [4,5]
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
    ('gb 5x5 128->1024 128x256', 4, 128, 1024, 5, 128, 256, 2),
    ('gb 5x5 128->512 256x512', 4, 128, 512, 5, 256, 512, 2),
    ('gb 5x5 128->2048 64x128', 4, 128, 2048, 5, 64, 128, 2),
    ('gb 5x5 128->4096 32x64', 4, 128, 4096, 5, 32, 64, 2),
    ('G up2 3x3 512->512 128x256', 4, 512, 512, 3, 128, 256, 1),
    ('G up1 3x3 512->512 64x128', 4, 512, 512, 3, 64, 128, 1),
    ('G up0 3x3 1024->1024 32x64', 4, 1024, 1024, 3, 32, 64, 1),
    ('G 3x3 1024->512 64x128', 4, 1024, 512, 3, 64, 128, 1),
    ('G 3x3 2048->1024 32x64', 4, 2048, 1024, 3, 32, 64, 1),
    ('G 3x3 512->256 128x256', 4, 512, 256, 3, 128, 256, 1),
    ('G 3x3 256->256 128x256', 4, 256, 256, 3, 128, 256, 1),
    ('dgrad 3x3 512->512 128x256', 4, 512, 512, 3, 128, 256, 1),
    ('dgrad 3x3 1024->512 64x128', 4, 1024, 512, 3, 64, 128, 1),
    ('dgrad 3x3 256->512 128x256', 4, 256, 512, 3, 128, 256, 1),
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
VERS = sys.argv[1].split(',') if len(sys.argv) > 1 else ['4', '5']
torch.manual_seed(0)
tot = {v: 0.0 for v in VERS}
totf = 0.0
for name, B, cin, cout, k, H, W, pad in shapes:
    x = torch.randn(B, cin, H, W, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(cout, cin, k, k, device='cuda', dtype=torch.bfloat16) /
         (cin * k * k) ** 0.5).contiguous(memory_format=CL)
    bias = torch.randn(cout, device='cuda', dtype=torch.float32)
    ref = F.leaky_relu(F.conv2d(x.float(), w.float(), bias, 1, pad), 0.2)
    flops = 2.0 * B * ref.shape[2] * ref.shape[3] * cout * cin * k * k
    errs = {}
    for v in VERS:
        os.environ['IMAGINAIRE_AMD_CONV_V'] = v
        y = ext.conv2d_mfma(x, w, bias, 1, 1, pad, pad, 1, 1, 0.2)
        errs[v] = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    ts = {v: [] for v in VERS}
    for rnd in range(3):
        for v in VERS:
            os.environ['IMAGINAIRE_AMD_CONV_V'] = v
            ts[v].append(timeit(lambda: ext.conv2d_mfma(x, w, bias, 1, 1, pad, pad, 1, 1, 0.2)))
    line = '%-30s' % name
    for v in VERS:
        t = min(ts[v])
        tot[v] += t
        line += ' | v%s %7.3f ms %5.0f TF/s err %.1e' % (v, t, flops / t / 1e9, errs[v])
    totf += flops
    for v in VERS[1:]:
        line += ' | v%s/v%s %.2fx' % (v, VERS[0], min(ts[VERS[0]]) / min(ts[v]))
    print(line, flush=True)
    for v in VERS:
        assert errs[v] < 2e-2, (name, v, errs[v])
os.environ.pop('IMAGINAIRE_AMD_CONV_V', None)
print('TOTAL ' + ' | '.join('v%s %.3f ms %.0f TF/s' % (v, tot[v], totf / tot[v] / 1e9)
                            for v in VERS), flush=True)
