"""Host-side cost per launch: MIOpen conv (fwd, fwd+bwd), rocBLAS mv and an
elementwise op, in PyTorch's default MIOpen mode and in benchmark mode.

    python scripts/probe/launch_overhead_probe.py [bench|nobench] [nhwc|nchw]
"""
import sys
import time

import torch
import torch.nn.functional as F

mode = sys.argv[1] if len(sys.argv) > 1 else 'nobench'
layout = sys.argv[2] if len(sys.argv) > 2 else 'nhwc'
torch.backends.cudnn.benchmark = mode == 'bench'
dev = 'cuda'
fmt = torch.channels_last if layout == 'nhwc' else torch.contiguous_format


def timeit(name, fn, n=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t_host = (time.perf_counter() - t0) / n * 1e3
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / n * 1e3
    print('%-44s %s/%s host %8.3f ms/call  wall %8.3f ms/call' % (name, mode, layout, t_host,
                                                               t_all), flush=True)


for (cin, cout, k, H, W) in [(512, 512, 3, 64, 128), (128, 1024, 5, 128, 256), (64, 3, 3, 256, 512)]:
    x = torch.randn(4, cin, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=fmt)
    w = (torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16) * 0.02).contiguous(
        memory_format=fmt)
    timeit('conv fwd %d->%d k%d %dx%d' % (cin, cout, k, H, W),
           lambda: F.conv2d(x, w, None, 1, k // 2))
    xg = x.detach().requires_grad_(True)
    wg = w.detach().requires_grad_(True)
    g = torch.randn(4, cout, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=fmt)

    def fb():
        y = F.conv2d(xg, wg, None, 1, k // 2)
        torch.autograd.grad(y, (xg, wg), g)
    timeit('conv fwd+bwd %d->%d k%d %dx%d' % (cin, cout, k, H, W), fb, n=20)
m = torch.randn(512, 4608, device=dev)
v = torch.randn(4608, device=dev)
timeit('mv 512x4608 fp32', lambda: torch.mv(m, v))
a = torch.randn(4, 512, 64, 128, device=dev)
timeit('add 4x512x64x128 fp32', lambda: a + a)
