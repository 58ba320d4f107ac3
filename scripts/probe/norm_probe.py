"""k1 SPADE norm kernels at the SPADE step shapes: time vs the bytes they must move."""
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


X = _ext.ext()
cl = torch.channels_last
for shape in ((4, 512, 128, 256), (4, 1024, 64, 128), (4, 256, 256, 512), (4, 2048, 16, 32)):
    x = torch.randn(*shape, device='cuda').to(torch.bfloat16).contiguous(memory_format=cl)
    gam = torch.randn_like(x)
    bet = torch.randn_like(x)
    cnt, mean, var, scale, shift = X.norm_stats(x, False, 1e-5, None, None, False)
    nb = x.numel() * 2
    ta = t(lambda: X.norm_apply(x, scale, shift, gam, bet, 0.2))
    ts = t(lambda: X.norm_stats(x, False, 1e-5, None, None, False))
    tc = t(lambda: x.clone())
    print('%s: stats %.3f ms (%.2f TB/s)  apply %.3f ms (%.2f TB/s, 4 passes)  clone %.3f ms' % (
        shape, ts, nb / ts / 1e9, ta, 4 * nb / ta / 1e9, tc))
