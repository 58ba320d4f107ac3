"""Run one k10 / k11 conv shape N times (target for rocprofv3 --pmc counter passes).

    python scripts/probe/conv_kernel_driver.py {fwd|wgrad|dgrad} B Cin Cout H W k [iters] [stride]

dgrad runs the stride-1 data gradient as k10 sees it: dy [B, Cout, H, W] convolved with the
flipped, transposed weight [Cin, Cout, k, k] (the narrow-N, wide-K GEMM of the SPADE convs).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402

mode = sys.argv[1]
B, cin, cout, H, W, k = (int(v) for v in sys.argv[2:8])
iters = int(sys.argv[8]) if len(sys.argv) > 8 else 20
st = int(sys.argv[9]) if len(sys.argv) > 9 else 1  # (fwd / wgrad only)
CL = torch.channels_last
pad = (k - 1) // 2
x = torch.randn(B, cin, H, W, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
w = (torch.randn(cout, cin, k, k, device='cuda', dtype=torch.bfloat16) * 0.02).contiguous(
    memory_format=CL)
Ho, Wo = (H + 2 * pad - k) // st + 1, (W + 2 * pad - k) // st + 1
g = torch.randn(B, cout, Ho, Wo, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
ext = _ext.ext()
wt = ext.conv_weight_flip_t(w, 1, 0, 0, 1) if mode == 'dgrad' else None
for _ in range(iters):
    if mode == 'fwd':
        ext.conv2d_mfma(x, w, None, st, st, pad, pad, 1, 1, 1.0)
    elif mode == 'dgrad':
        ext.conv2d_mfma(g, wt, None, 1, 1, k - 1 - pad, k - 1 - pad, 1, 1, 1.0)
    else:
        ext.conv2d_wgrad_mfma(g, x, k, k, st, st, pad, pad, 1, 1)
torch.cuda.synchronize()
print('done', mode, 'variant', ext.conv_last_variant() if mode != 'wgrad' else '-')
