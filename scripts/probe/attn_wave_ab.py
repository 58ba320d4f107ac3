"""k16 at the few-shot recipe shape: the 8-wave grid threshold (IMAGINAIRE_AMD_ATTN_MIN_WG, read
per call) A/B, forward and forward + backward, interleaved.

    python scripts/probe/attn_wave_ab.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import attention as A  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


torch.manual_seed(0)
B, Lq, Lk, d, dv = 3, 16384, 32768, 128, 258
q = torch.randn(B, Lq, d, device='cuda').to(torch.bfloat16)
k = torch.randn(B, Lk, d, device='cuda').to(torch.bfloat16)
v = torch.randn(B, Lk, dv, device='cuda').to(torch.bfloat16)
qg, kg, vg = (t.clone().requires_grad_(True) for t in (q, k, v))
go = torch.randn(B, Lq, dv, device='cuda').to(torch.bfloat16)
res = {}
for rnd in range(3):
    for mw in ('512', '256', '128'):
        os.environ['IMAGINAIRE_AMD_ATTN_MIN_WG'] = mw
        f = timeit(lambda: A.fused_attention(q, k, v))
        fb = timeit(lambda: A.fused_attention(qg, kg, vg).backward(go))
        res.setdefault(mw, []).append((f, fb))
for mw, r in res.items():
    print('min_wg %s: fwd %.3f ms  fwd+bwd %.3f ms' % (mw, min(x[0] for x in r),
                                                       min(x[1] for x in r)), flush=True)
