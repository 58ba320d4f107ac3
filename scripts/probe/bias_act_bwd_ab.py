"""k2 bias + activation backward (channels-last): 4 rows per trip with their loads issued first
(IMAGINAIRE_AMD_BIASACT_UNROLL=4, default) vs one row (1), on SPADE-step shapes, interleaved,
minimum of three rounds; outputs must match bitwise (same summation order).

    python scripts/probe/bias_act_bwd_ab.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402

E = _ext.ext()
CL = torch.channels_last
SHAPES = [((4, 1024, 64, 128), 0.2), ((4, 512, 128, 256), 0.2), ((4, 256, 256, 512), 0.2),
          ((8, 128, 128, 256), 0.2), ((4, 2048, 64, 128), 1.0), ((4, 1024, 128, 256), 1.0),
          ((4, 512, 32, 64), 0.2)]


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


torch.manual_seed(0)
for shape, slope in SHAPES:
    y = torch.randn(shape, device='cuda').to(torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(shape, device='cuda').to(torch.bfloat16).contiguous(memory_format=CL)
    res, outs = {}, {}
    for rnd in range(3):
        for u in ('4', '1'):
            os.environ['IMAGINAIRE_AMD_BIASACT_UNROLL'] = u
            d = dy.clone() if slope == 1.0 else dy
            res.setdefault(u, []).append(timeit(lambda: E.bias_act_bwd(y, d, slope)))
            outs[u] = [t.float().clone() for t in E.bias_act_bwd(y, dy.clone(), slope)]
    same = all(torch.equal(a, b) for a, b in zip(outs['4'], outs['1']))
    nbytes = y.numel() * 2 * (3 if slope != 1.0 else 1)
    t4, t1 = min(res['4']), min(res['1'])
    print('%-22s slope %.1f  unroll4 %.1f us (%.2f TB/s)  unroll1 %.1f us (%.2f TB/s)  %.2fx  '
          'bitwise %s' % (shape, slope, t4 * 1e3, nbytes / t4 / 1e9, t1 * 1e3, nbytes / t1 / 1e9,
                          t1 / t4, same), flush=True)
os.environ.pop('IMAGINAIRE_AMD_BIASACT_UNROLL', None)
