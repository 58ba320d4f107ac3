"""k11 five-tap weight gradients: the 64 x 64 multi-tap tile (default) vs the 128 x 64 tile with
tap-pipelined fragment reads (IMAGINAIRE_AMD_WGRAD_MT5=128, read per call), on the SPADE-step
5x5 shapes; interleaved in one process, values checked against fp32 torch.

    python scripts/probe/wgrad_mt5_probe.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402

CL = torch.channels_last
shapes = [
    # name, B, cin, cout, H, W
    ('gb 128->1024 128x256', 4, 128, 1024, 128, 256),
    ('gb 128->512 256x512', 4, 128, 512, 256, 512),
    ('gb 128->2048 64x128', 4, 128, 2048, 64, 128),
    ('gb 128->4096 32x64', 4, 128, 4096, 32, 64),
    ('shared 192->128 128x256', 4, 192, 128, 128, 256),
    ('shared 192->128 256x512', 4, 192, 128, 256, 512),
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
torch.manual_seed(0)
tot = {'64': 0.0, '128': 0.0}
for name, B, cin, cout, H, W in shapes:
    x = torch.randn(B, cin, H, W, device='cuda').to(torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(B, cout, H, W, device='cuda').to(torch.bfloat16).contiguous(memory_format=CL)
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, 5, 5), dy.float(), 1, 2)
    flops = 2.0 * B * H * W * cout * cin * 25
    row = []
    for v in ('64', '128'):
        os.environ['IMAGINAIRE_AMD_WGRAD_MT5'] = v
        fn = lambda: ext.conv2d_wgrad_mfma(dy, x, 5, 5, 1, 1, 2, 2, 1, 1)  # noqa: E731
        g = fn()
        err = float((g.float() - ref).abs().max()) / float(ref.abs().max())
        t = timeit(fn)
        tot[v] += t
        row.append('%s: %.3f ms %5.0f TF/s err %.1e' % (v, t, flops / t / 1e9, err))
    os.environ.pop('IMAGINAIRE_AMD_WGRAD_MT5')
    print('%-26s %s' % (name, ' | '.join(row)), flush=True)
print('TOTAL 64x64 %.3f ms | 128x64 %.3f ms | %.2fx' % (tot['64'], tot['128'],
                                                      tot['64'] / tot['128']))
