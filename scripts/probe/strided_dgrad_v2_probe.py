"""Strided data gradients: all phases in one k10 launch stored in place (conv2d_dgrad_strided)
vs per-phase launches + scatter (round 2-3 path), on the SPADE-step shapes, interleaved in one
process (cdna guide rule 24).

    python scripts/probe/strided_dgrad_v2_probe.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import conv  # noqa: E402

CL = torch.channels_last
shapes = [  # dy shape [B, Cout, Ho, Wo], weight [Cout, Cin, k, k], stride, pad
    ((8, 512, 32, 64), (512, 256, 4, 4), 2, 1),
    ((8, 512, 16, 32), (512, 512, 4, 4), 2, 1),
    ((8, 512, 8, 16), (512, 512, 4, 4), 2, 1),
    ((4, 128, 128, 256), (128, 192, 4, 4), 2, 1),
    ((8, 256, 64, 128), (256, 128, 4, 4), 2, 1),
    ((8, 1024, 16, 32), (1024, 512, 3, 3), 2, 1),
    ((8, 512, 32, 64), (512, 256, 3, 3), 2, 1),
    ((4, 1024, 8, 16), (1024, 1024, 3, 3), 2, 1),
    ((4, 256, 64, 128), (256, 128, 3, 3), 2, 1),
]


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


torch.manual_seed(0)
tot = [0.0, 0.0]
for dys, ws, s, p in shapes:
    dy = torch.randn(dys, device='cuda').to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(ws, device='cuda') * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    H = (dys[2] - 1) * s - 2 * p + ws[2]
    W = (dys[3] - 1) * s - 2 * p + ws[3]
    fl = 2.0 * dy.numel() * ws[1] * ws[2] * ws[3]
    res = {}
    outs = {}
    for mode in (0, 1):
        conv._STRIDED_ONE_LAUNCH = bool(mode)
        outs[mode] = conv._strided_dgrad(dy, w, H, W, s, (p, p))
    err = ((outs[0].float() - outs[1].float()).abs().max() / outs[0].float().abs().max()).item()
    ts = {0: [], 1: []}
    for _ in range(3):
        for mode in (0, 1):
            conv._STRIDED_ONE_LAUNCH = bool(mode)
            ts[mode].append(timeit(lambda: conv._strided_dgrad(dy, w, H, W, s, (p, p))))
    t0, t1 = min(ts[0]), min(ts[1])
    tot[0] += t0
    tot[1] += t1
    print('dy %-20s w %-20s s%d | phases+scatter %.3f ms %4.0f TF/s | one launch %.3f ms %4.0f '
          'TF/s | %.2fx | diff %.1e' % (dys, ws, s, t0, fl / t0 / 1e9, t1, fl / t1 / 1e9, t0 / t1,
                                        err), flush=True)
    assert err < 1e-2
print('TOTAL phases+scatter %.3f ms | one launch %.3f ms | %.2fx' % (tot[0], tot[1], tot[0] / tot[1]))
