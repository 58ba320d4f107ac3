"""FlowNetC correlation forward: LDS-tiled VALU (k6), one-wave MFMA (k6m) and the diagonal
multi-wave MFMA kernel (image-2 strip staged once per row, the default), bf16.

    python scripts/probe/corr_probe.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402
from imaginaire_amd.ops.flownet_ops import correlation_reference  # noqa: E402

ext = _ext.ext()
CL = torch.channels_last
for N, C, H, W in ((2, 256, 64, 128), (4, 256, 64, 128), (4, 256, 32, 64)):
    a = torch.randn(N, C, H, W, device='cuda').to(torch.bfloat16).contiguous(memory_format=CL)
    b = torch.randn(N, C, H, W, device='cuda').to(torch.bfloat16).contiguous(memory_format=CL)
    res = {}
    for tag, env, dg in (('valu', '0', '0'), ('mfma', '1', '0'), ('diag', '1', '1')):
        os.environ['IMAGINAIRE_AMD_CORR_MFMA'] = env
        os.environ['IMAGINAIRE_AMD_CORR_DIAG'] = dg
        y = ext.correlation_forward(a, b, 20, 1, 20, 1, 2)
        for _ in range(3):
            ext.correlation_forward(a, b, 20, 1, 20, 1, 2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            ext.correlation_forward(a, b, 20, 1, 20, 1, 2)
        torch.cuda.synchronize()
        res[tag] = ((time.perf_counter() - t0) / 20 * 1e3, y.float())
    ref = correlation_reference(a.float(), b.float(), 20, 1, 20, 1, 2)
    err = max((res[k][1] - ref).abs().max().item() for k in res)
    flops = 2.0 * N * H * W * 441 * C
    print('corr N=%d C=%d %dx%d  valu %.3f ms | mfma %.3f ms (%.0f TF/s) | diag %.3f ms '
          '(%.0f TF/s, x%.2f vs mfma)  max err %.2e' % (
              N, C, H, W, res['valu'][0], res['mfma'][0], flops / res['mfma'][0] / 1e9,
              res['diag'][0], flops / res['diag'][0] / 1e9, res['mfma'][0] / res['diag'][0], err),
          flush=True)
