"""The SPADE-step convs whose grids cannot fill the chip (few output pixels or channels):
k10 v1 vs v4 and split-K factors (IMAGINAIRE_AMD_CONV_V / IMAGINAIRE_AMD_CONV_SPLITK, both read
per call), interleaved in one process.

    python scripts/probe/conv_small_probe.py
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
    ('mlp_shared 192->128 5x5 16x32', 4, 192, 128, 5, 16, 32, 2),
    ('mlp_shared 192->128 5x5 32x64', 4, 192, 128, 5, 32, 64, 2),
    ('mlp_shared 192->128 5x5 64x128', 4, 192, 128, 5, 64, 128, 2),
    ('D 512->512 3x3 32x64', 4, 512, 512, 3, 32, 64, 1),
    ('vgg 64->64 3x3 256x512', 4, 64, 64, 3, 256, 512, 1),
    ('vgg 256->256 3x3 64x128', 4, 256, 256, 3, 64, 128, 1),
    ('gb 128->4096 5x5 16x32', 4, 128, 4096, 5, 16, 32, 2),
]


def timeit(fn, iters=30):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


ext = _ext.ext()
torch.manual_seed(0)
configs = [('1', None), ('4', None), ('1', '4'), ('1', '8'), ('1', '16'), ('4', '4'), ('4', '8'),
           ('4', '16')]
for name, B, cin, cout, k, H, W, pad in shapes:
    x = torch.randn(B, cin, H, W, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(cout, cin, k, k, device='cuda', dtype=torch.bfloat16) /
         (cin * k * k) ** 0.5).contiguous(memory_format=CL)
    bias = torch.randn(cout, device='cuda', dtype=torch.float32)
    ref = F.leaky_relu(F.conv2d(x.float(), w.float(), bias, 1, pad), 0.2)
    flops = 2.0 * B * H * W * cout * cin * k * k
    row = []
    for ver, sk in configs:
        os.environ['IMAGINAIRE_AMD_CONV_V'] = ver
        if sk is None:
            os.environ.pop('IMAGINAIRE_AMD_CONV_SPLITK', None)
        else:
            os.environ['IMAGINAIRE_AMD_CONV_SPLITK'] = sk
        fn = lambda: ext.conv2d_mfma(x, w, bias, 1, 1, pad, pad, 1, 1, 0.2, 1, -1)  # noqa: E731
        y = fn()
        err = float((y.float() - ref).abs().max()) / max(1e-6, float(ref.abs().max()))
        t = timeit(fn)
        row.append('v%s/S%s %.3f ms %4.0f TF/s%s' % (ver, sk or 'auto', t, flops / t / 1e9,
                                                    '' if err < 2e-2 else ' ERR %.2g' % err))
    os.environ.pop('IMAGINAIRE_AMD_CONV_V', None)
    os.environ.pop('IMAGINAIRE_AMD_CONV_SPLITK', None)
    print('%-34s %s' % (name, ' | '.join(row)), flush=True)
