"""k16 backward alone at the few-shot recipe shape: 8- vs 4-wave workgroups for the dK/dV and the
dQ kernels separately (IMAGINAIRE_AMD_ATTN_DKV_MIN_WG / IMAGINAIRE_AMD_ATTN_DQ_MIN_WG, read per
call), interleaved, minimum of three rounds; each variant's gradients are checked against the
default's.

    python scripts/probe/attn_bwd_ab.py [--default-only | --dq-gemm | --gemm-waves]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402

B, Lq, Lk, d, dv = 3, 16384, 32768, 128, 288  # 258 value channels, padded as fused_attention does
scale = d ** -0.5
torch.manual_seed(0)
q = torch.randn(B, Lq, d, device='cuda').to(torch.bfloat16)
k = torch.randn(B, Lk, d, device='cuda').to(torch.bfloat16)
v = torch.randn(B, Lk, dv, device='cuda').to(torch.bfloat16)
go = torch.randn(B, Lq, dv, device='cuda').to(torch.bfloat16)
E = _ext.ext()
o, lse = E.attention_fwd(q, k, v, scale)


def bwd():
    return E.attention_bwd(q, k, v, o, lse, go, scale)


def timeit(iters=10):
    bwd()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        bwd()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


BIG = '100000000'
VARIANTS = {'dkv8 dq8 (default)': (None, None), 'dkv4 dq8': (BIG, None),
            'dkv8 dq4': (None, BIG), 'dkv4 dq4': (BIG, BIG)}
if '--dq-gemm' in sys.argv:  # dQ from the stored dS^T by one GEMM vs the dQ kernel
    VARIANTS = {'dq gemm (default)': (None, None, '1'), 'dq kernel': (None, None, '0')}
if '--gemm-waves' in sys.argv:  # the GEMM path with 8- vs 4-wave dK/dV (+dS^T) workgroups
    VARIANTS = {'gemm dkv8': (None, None, '1'), 'gemm dkv4': (BIG, None, '1')}
if '--default-only' in sys.argv:  # for a per-kernel rocprofv3 breakdown of the default
    VARIANTS = {'dkv8 dq8 (default)': (None, None)}


def setenv(a, b, gemm=None):
    for var, val in (('IMAGINAIRE_AMD_ATTN_DKV_MIN_WG', a), ('IMAGINAIRE_AMD_ATTN_DQ_MIN_WG', b),
                     ('IMAGINAIRE_AMD_ATTN_DQ_GEMM', gemm)):
        if val is None:
            os.environ.pop(var, None)
        else:
            os.environ[var] = val


setenv(None, None, '0')
ref = [t.float() for t in bwd()]  # the dQ kernel path
flops = 2 * B * Lq * Lk * (2 * d + 2 * dv + d)  # S, dP, dV, dK, dQ  (recompute S: + d)
res = {}
for rnd in range(3):
    for name, vs in VARIANTS.items():
        setenv(*vs)
        res.setdefault(name, []).append(timeit())
for name, vs in VARIANTS.items():
    setenv(*vs)
    got = bwd()
    err = max(float((g.float() - r).abs().max() / r.abs().max()) for g, r in zip(got, ref))
    t = min(res[name])
    print('%-20s bwd %.3f ms  (%.0f TF/s)  max rel diff vs dQ-kernel path %.2e'
          % (name, t, flops / t / 1e9, err), flush=True)
setenv(None, None)
