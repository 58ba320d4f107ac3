"""k10 variants on the narrow-N (N = Cin = 128) / wide-K data gradients of the SPADE gamma|beta
convs and a few other step shapes: v1 BM=128 (default), v1 BM=256, v3 512x128."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from imaginaire_amd.ops import _ext  # noqa: E402


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
    X = _ext.ext()
    cl = torch.channels_last
    # (B, Cin_of_dgrad_input(=Cout of fwd), H, W, Cout_of_dgrad(=Cin of fwd), k)
    shapes = [(4, 1024, 128, 256, 128, 5), (4, 2048, 64, 128, 128, 5), (4, 4096, 32, 64, 128, 5),
              (4, 512, 128, 256, 512, 3), (4, 1024, 32, 64, 1024, 3), (4, 128, 128, 256, 1024, 5)]
    variants = [('v1 bm128', {'IMAGINAIRE_AMD_CONV_V': '1'}),
                ('v1 bm256', {'IMAGINAIRE_AMD_CONV_V': '1', 'IMAGINAIRE_AMD_CONV_BM': '256'}),
                ('v3', {'IMAGINAIRE_AMD_CONV_V': '3'}), ('auto', {})]
    for B, ci, H, W, co, k in shapes:
        x = torch.randn(B, ci, H, W, device='cuda').to(torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(co, ci, k, k, device='cuda') * 0.02).to(torch.bfloat16).contiguous(memory_format=cl)
        fl = 2.0 * B * H * W * co * ci * k * k
        row = []
        for name, env in variants:
            for key in ('IMAGINAIRE_AMD_CONV_V', 'IMAGINAIRE_AMD_CONV_BM'):
                os.environ.pop(key, None)
            os.environ.update(env)
            ms = t(lambda: X.conv2d_mfma(x, w, None, 1, 1, k // 2, k // 2, 1, 1, 1.0, 1))
            row.append('%s %.3f ms %4.0f TF/s' % (name, ms, fl / ms / 1e9))
        print('[%d,%d,%d,%d]x[%d,%d,%d,%d]: ' % (B, ci, H, W, co, ci, k, k) + ' | '.join(row))


if __name__ == '__main__':
    main()
