"""Strided-conv data gradient: k10 phase convolutions vs MIOpen backward-data on the SPADE
discriminator shapes (times per call, max error vs fp32)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from imaginaire_amd.ops import conv as C  # noqa: E402


def t(fn, n=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n


def main():
    cl = torch.channels_last
    # (B, Cin, H, W, Cout, K, s, p): x [B, Cin, H, W] -> dy [B, Cout, Ho, Wo]
    shapes = [(4, 192, 256, 512, 128, 4, 2, 1), (8, 128, 128, 256, 256, 4, 2, 1),
              (8, 256, 64, 128, 512, 4, 2, 1), (8, 512, 32, 64, 1024, 3, 2, 1),
              (8, 128, 128, 256, 256, 3, 2, 1), (8, 512, 16, 32, 512, 4, 2, 1),
              (8, 256, 64, 128, 512, 3, 2, 1)]
    for B, ci, H, W, co, k, s, p in shapes:
        x = torch.randn(B, ci, H, W, device='cuda').to(torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(co, ci, k, k, device='cuda') / (ci * k * k) ** 0.5).to(
            torch.bfloat16).contiguous(memory_format=cl)
        y = F.conv2d(x, w, None, s, p)
        dy = torch.randn_like(y).contiguous(memory_format=cl)
        ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, (s, s),
                                                  (p, p), (1, 1), False, [0, 0], 1,
                                                  [True, False, False])[0]
        got = C._strided_dgrad(dy, w, H, W, s, (p, p))
        err = float((got.float() - ref).abs().max()) / max(1e-6, float(ref.abs().max()))
        tm = t(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, (s, s), (p, p), (1, 1), False, [0, 0], 1, [True, False, False]))
        tk = t(lambda: C._strided_dgrad(dy, w, H, W, s, (p, p)))
        fl = 2.0 * B * y.shape[2] * y.shape[3] * co * ci * k * k
        print('dx [%d,%d,%d,%d] w [%d,%d,%d,%d] s%d: MIOpen %.3f ms (%.0f TF/s)  k10 phases %.3f ms '
              '(%.0f TF/s)  rel err %.2e' % (B, ci, H, W, co, ci, k, k, s, tm, fl / tm / 1e9, tk,
                                             fl / tk / 1e9, err))


if __name__ == '__main__':
    main()
