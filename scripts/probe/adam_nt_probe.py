"""A/B of the multi-tensor Adam kernel with plain vs non-temporal fp32 loads / stores
(IMAGINAIRE_AMD_ADAM_NT / IMAGINAIRE_AMD_EMA_NT, read once per process: run this script once per setting).

SPADE-recipe-sized parameter set: 415M fp32 parameters in 400 tensors (fp32 grads, a bf16
shadow on the conv weights), i.e. the optimizer traffic of one bench step. Prints ms per
mt_adam call and the effective HBM bandwidth (16 B read + 12 B written per parameter, + 2 B for
shadowed ones).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402


def main():
    torch.manual_seed(0)
    dev = torch.device('cuda', 0)
    sizes = []
    total, target = 0, 415_000_000
    i = 0
    while total < target:
        n = [2_359_296, 1_179_648, 589_824, 147_456, 4_096, 512][i % 6]
        sizes.append(n)
        total += n
        i += 1
    p = [torch.randn(n, device=dev) for n in sizes]
    g = [torch.randn(n, device=dev) * 1e-3 for n in sizes]
    m = [torch.zeros(n, device=dev) for n in sizes]
    v = [torch.zeros(n, device=dev) for n in sizes]
    sh = [torch.empty(n, device=dev, dtype=torch.bfloat16) if n > 4096 else
          torch.empty(0, device=dev, dtype=torch.bfloat16) for n in sizes]
    nshadow = sum(n for n in sizes if n > 4096)
    ext = _ext.ext()
    for s in range(1, 4):
        ext.mt_adam(p, g, m, v, sh, 1e-4, 0.0, 0.999, 1e-8, s, 0.0, False, 1.0, None)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    iters = 20
    e0.record()
    for s in range(4, 4 + iters):
        ext.mt_adam(p, g, m, v, sh, 1e-4, 0.0, 0.999, 1e-8, s, 0.0, False, 1.0, None)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    nbytes = 28 * total + 2 * nshadow
    print('adam NT=%s: %d params in %d tensors: %.3f ms/call, %.2f TB/s effective' % (
        os.environ.get('IMAGINAIRE_AMD_ADAM_NT', '1'), total, len(sizes), ms,
        nbytes / ms / 1e9))
    # EMA of the same set (IMAGINAIRE_AMD_EMA_NT): 8 B read + 4 B written per parameter
    avg = [torch.zeros(n, device=dev) for n in sizes]
    for _ in range(3):
        ext.mt_ema(avg, p, 0.999, None, None, 0)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        ext.mt_ema(avg, p, 0.999, None, None, 0)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    print('ema NT=%s: %.3f ms/call, %.2f TB/s effective' % (
        os.environ.get('IMAGINAIRE_AMD_EMA_NT', '1'), ms, 12 * total / ms / 1e9))


if __name__ == '__main__':
    main()
