"""Time the pieces of the tap-split conv (SPADE conv_img shape) against the k10 direct conv."""
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


def main():
    X = _ext.ext()
    B, cin, H, W, k, cout = 4, 256, 256, 512, 5, 3
    cz = 128
    cl = torch.channels_last
    x = torch.randn(B, cin, H, W, device='cuda').to(torch.bfloat16).contiguous(memory_format=cl)
    wz = (torch.randn(cz, cin, 1, 1, device='cuda') * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
    w64 = (torch.randn(64, cin, k, k, device='cuda') * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
    bias = torch.zeros(cout, device='cuda')
    z = X.conv2d_mfma(x, wz, None, 1, 1, 0, 0, 1, 1, 1.0, 1)
    y = X.conv_tap_sum(z, bias, cout, k, k, 2, 2, 1, 1)
    dy = torch.randn_like(y.float()).to(torch.bfloat16)
    print('k10 direct 5x5 (Cout pad 64): %.3f ms' % t(lambda: X.conv2d_mfma(x, w64, None, 1, 1, 2, 2, 1, 1, 1.0, 1)))
    print('k10 1x1 -> Z (N=128, K=256): %.3f ms' % t(lambda: X.conv2d_mfma(x, wz, None, 1, 1, 0, 0, 1, 1, 1.0, 1)))
    print('tap_sum: %.3f ms' % t(lambda: X.conv_tap_sum(z, bias, cout, k, k, 2, 2, 1, 1)))
    print('tap_gather: %.3f ms' % t(lambda: X.conv_tap_gather(dy, cz, k, k, 2, 2, 1, 1, H, W)))
    dz = X.conv_tap_gather(dy, cz, k, k, 2, 2, 1, 1, H, W)
    wzt = wz.view(cz, cin).t().contiguous().view(cin, cz, 1, 1)
    print('k10 1x1 dgrad (N=256, K=128): %.3f ms' % t(lambda: X.conv2d_mfma(dz, wzt, None, 1, 1, 0, 0, 1, 1, 1.0, 1)))
    print('k11 1x1 wgrad: %.3f ms' % t(lambda: X.conv2d_wgrad_mfma(dz, x, 1, 1, 1, 1, 0, 0, 1, 1, 75, cin, False, 1)))
    print('copy x (268 MB r+w): %.3f ms' % t(lambda: x.clone()))


if __name__ == '__main__':
    main()
