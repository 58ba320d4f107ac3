"""NHWC reflect-pad kernel timing vs a plain copy of the same bytes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from imaginaire_amd.ops import _ext  # noqa: E402


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n


for shape, p in (((2, 1024, 32, 64), 1), ((2, 64, 512, 1024), 3), ((16, 256, 64, 64), 1),
                 ((16, 64, 256, 256), 3)):
    x = torch.randn(*shape, device='cuda').to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = _ext.ext().pad_nhwc_fwd(x, p, p, p, p, 0)
    tf = t(lambda: _ext.ext().pad_nhwc_fwd(x, p, p, p, p, 0))
    tb = t(lambda: _ext.ext().pad_nhwc_bwd(y, shape[2], shape[3], p, p, p, p, 0))
    tc = t(lambda: y.clone())
    gb = (x.numel() + y.numel()) * 2 / 1e9
    print('%s pad %d: fwd %.3f ms (%.2f TB/s)  bwd %.3f ms  clone(out) %.3f ms' % (
        shape, p, tf, gb / tf, tb, tc))
