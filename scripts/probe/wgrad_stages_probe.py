"""A/B the k11 weight-gradient pipeline depth (IMAGINAIRE_AMD_WGRAD_STAGES = 2 | 3) in ONE
process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24), on the SPADE-step shapes
(profiles/spade_step_conv_log_mi355x.txt), with an fp32 reference check of each variant."""
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
    ('G 3x3 1024->1024 32x64', 4, 1024, 1024, 3, 32, 64),
    ('head 3x3 2048->2048 16x32', 4, 2048, 2048, 3, 16, 32),
    ('gb 5x5 128->4096 32x64', 4, 128, 4096, 5, 32, 64),
    ('gb 5x5 128->4096 16x32', 4, 128, 4096, 5, 16, 32),
    ('gb 5x5 128->2048 64x128', 4, 128, 2048, 5, 64, 128),
]
for name, B, cin, cout, k, H, W in shapes:
    pad = k // 2
    torch.manual_seed(0)
    x = torch.randn(B, cin, H, W, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(B, cout, H, W, device='cuda', dtype=torch.bfloat16).contiguous(
        memory_format=CL)
    flops = 2.0 * B * H * W * cout * cin * k * k
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, k, k), dy.float(), padding=pad)
    res = {v: [] for v in ('2', '3')}
    errs = {}
    for rnd in range(5):
        for v in res:
            os.environ['IMAGINAIRE_AMD_WGRAD_STAGES'] = v

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
    print('%-28s ' % name + ' | '.join('nst%s %6.3f ms %5.0f TF/s err %.1e' % (
        v, min(t), flops / min(t) / 1e9, errs[v]) for v, t in res.items()) +
        ' | 3/2 %.2fx' % (min(res['2']) / min(res['3'])), flush=True)
