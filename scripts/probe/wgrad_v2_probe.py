"""A/B the k11 weight-gradient kernels in ONE process, interleaved rounds (cdna_hip_programming.md
§5.4 rule 24): v2 (one wave per SIMD, 64 x 64 x KW-tap accumulators per wave) vs the round-2
kernels (IMAGINAIRE_AMD_WGRAD_V2=0: multi-tap 2-waves-per-SIMD / one-tap), on the SPADE-step
shapes (profiles/spade_step_conv_log_mi355x.txt), each checked against fp32 autograd.

    python scripts/probe/wgrad_v2_probe.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402

ext = _ext.ext()
CL = torch.channels_last
# (name, B, Cin, Cout, k, H, W)
shapes = [
    ('gb 5x5 128->1024 128x256', 4, 128, 1024, 5, 128, 256),
    ('G 3x3 512->512 128x256', 4, 512, 512, 3, 128, 256),
    ('mlp 5x5 192->128 128x256', 4, 192, 128, 5, 128, 256),
    ('gb 5x5 128->2048 64x128', 4, 128, 2048, 5, 64, 128),
    ('G 3x3 1024->1024 32x64', 4, 1024, 1024, 3, 32, 64),
    ('G 3x3 512->512 64x128', 4, 512, 512, 3, 64, 128),
    ('head 3x3 2048->2048 16x32', 4, 2048, 2048, 3, 16, 32),
    ('gb 5x5 128->4096 32x64', 4, 128, 4096, 5, 32, 64),
    ('gb 5x5 128->4096 16x32', 4, 128, 4096, 5, 16, 32),
    ('G 3x3 1024->2048 16x32', 4, 1024, 2048, 3, 16, 32),
    ('mlp 5x5 192->128 64x128', 4, 192, 128, 5, 64, 128),
]
only = os.environ.get('ONLY')
for name, B, cin, cout, k, H, W in shapes:
    if only and only not in name:
        continue
    pad = k // 2
    torch.manual_seed(0)
    x = torch.randn(B, cin, H, W, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(B, cout, H, W, device='cuda', dtype=torch.bfloat16).contiguous(
        memory_format=CL)
    flops = 2.0 * B * H * W * cout * cin * k * k
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, k, k), dy.float(), padding=pad)
    res = {v: [] for v in ('old', 'v2')}
    errs = {}
    for rnd in range(5):
        for v in res:
            os.environ['IMAGINAIRE_AMD_WGRAD_V2'] = 'force' if v == 'v2' else '0'

            def run():
                return ext.conv2d_wgrad_mfma(dy, x, k, k, 1, 1, pad, pad, 1, 1, -1, -1, False, 1)
            g = run()
            if rnd == 0:
                errs[v] = float((g.float() - ref).norm() / ref.norm())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                run()
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / 10 * 1e3)
    os.environ.pop('IMAGINAIRE_AMD_WGRAD_V2', None)
    print('%-28s ' % name + ' | '.join('%s %6.3f ms %5.0f TF/s err %.1e' % (
        v, min(t), flops / min(t) / 1e9, errs[v]) for v, t in res.items()) +
        ' | v2/old %.2fx' % (min(res['old']) / min(res['v2'])), flush=True)
