"""A/B the k10 main-loop schedule variants (IMAGINAIRE_AMD_CONV_VAR) in ONE process,
interleaved rounds (cdna_hip_programming.md §5.4 rule 24), on the SPADE-step shapes."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402

ext = _ext.ext()
CL = torch.channels_last
shapes = [
    ('up1 3x3 512->512 64x128', 4, 512, 512, 3, 64, 128),
    ('up3 3x3 128->128 256x512', 4, 128, 128, 3, 256, 512),
    ('mlp 5x5 192->128 256x512', 4, 192, 128, 5, 256, 512),
    ('gb 5x5 128->1024 128x256', 4, 128, 1024, 5, 128, 256),
    ('gb 5x5 128->512 256x512', 4, 128, 512, 5, 256, 512),
]
for name, B, cin, cout, k, H, W in shapes:
    pad = k // 2
    x = torch.randn(B, cin, H, W, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(cout, cin, k, k, device='cuda', dtype=torch.bfloat16) * 0.02).contiguous(
        memory_format=CL)
    flops = 2.0 * B * H * W * cout * cin * k * k
    res = {v: [] for v in ('0', '1', '2')}
    ref = None
    for rnd in range(5):
        for v in res:
            os.environ['IMAGINAIRE_AMD_CONV_VAR'] = v
            y = ext.conv2d_mfma(x, w, None, 1, 1, pad, pad, 1, 1, 1.0)
            if ref is None:
                ref = y.clone()
            assert torch.equal(y, ref), 'variant %s differs' % v
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                ext.conv2d_mfma(x, w, None, 1, 1, pad, pad, 1, 1, 1.0)
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / 10 * 1e3)
    print('%-28s ' % name + ' | '.join('var%s %6.3f ms %5.0f TF/s' % (
        v, min(t), flops / min(t) / 1e9) for v, t in res.items()), flush=True)
