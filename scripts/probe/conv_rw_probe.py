"""Row-window k10 tile (IMAGINAIRE_AMD_CONV_V=6) vs the v1 tile (=1) on the recipe shapes the
v4 / v5 tiles do not take: time per call and TF/s (useful FLOPs of the unpadded conv).

    python scripts/probe/conv_rw_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402

X = _ext.ext()
CL = torch.channels_last
# name, B, Cin, Cout, H, W, KH, KW, stride, pad
SHAPES = [
    ('vid2vid 64ch 3x3 @512x1024', 2, 64, 64, 512, 1024, 3, 3, 1, 1),
    ('vid2vid 32ch 3x3 @512x1024 (Cin 32)', 2, 32, 64, 512, 1024, 3, 3, 1, 1),
    ('vid2vid D 4x4 s2 @512x1024', 4, 64, 64, 512, 1024, 4, 4, 2, 1),
    ('vid2vid 1x1 64->64 @512x1024', 2, 64, 64, 512, 1024, 1, 1, 1, 0),
    ('vid2vid 1x1 64->128 @512x1024', 2, 64, 128, 512, 1024, 1, 1, 1, 0),
    ('vid2vid 1x1 32->64 (Cin 32)', 2, 32, 64, 512, 1024, 1, 1, 1, 0),
    ('MUNIT stem 7x7 (Cin 3->64 padded) @256', 16, 64, 64, 262, 262, 7, 7, 1, 0),
    ('MUNIT dec 5x5 128->64 @256', 16, 128, 64, 260, 260, 5, 5, 1, 0),
    ('MUNIT down 4x4 s2 64->128', 16, 64, 128, 258, 258, 4, 4, 2, 0),
    ('MUNIT down 4x4 s2 128->256', 16, 128, 256, 130, 130, 4, 4, 2, 0),
    ('MUNIT D 4x4 s2 64->64 @256', 16, 64, 64, 256, 256, 4, 4, 2, 1),
    ('pix2pixHD stem 7x7 @512x1024', 2, 64, 64, 518, 1030, 7, 7, 1, 0),
    ('fs 7x7 s2 64->64 @512', 3, 64, 64, 512, 512, 7, 7, 2, 3),
    ('fs 3x3 s2 256->512 @64', 3, 256, 512, 64, 64, 3, 3, 2, 1),
    ('fs 3x3 s2 64->64 @512', 3, 64, 64, 512, 512, 3, 3, 2, 1),
    ('fs 32ch 3x3 @512 (Cin 32)', 3, 32, 64, 512, 512, 3, 3, 1, 1),
    ('SPADE D 4x4 s2 192->128 @256x512', 8, 192, 128, 256, 512, 4, 4, 2, 1),
    ('SPADE 1x1 512->256 @128x256', 4, 512, 256, 128, 256, 1, 1, 1, 0),
    ('D 4x4 s1 p2 512->512 @7x15', 8, 512, 512, 7, 15, 4, 4, 1, 2),
    ('D 4x4 s2 512->512 @16x32', 8, 512, 512, 16, 32, 4, 4, 2, 1),
    # round 6: odd-width data gradients of reflect-padded 3x3 convs (dy 64 wide -> dx 66)
    ('MUNIT res dgrad 256 @64 -> 66', 16, 256, 256, 64, 64, 3, 3, 1, 2),
    ('FUNIT res dgrad 1024 @16 -> 18', 16, 1024, 1024, 16, 16, 3, 3, 1, 2),
    ('FUNIT res dgrad 512 @32 -> 34', 16, 512, 512, 32, 32, 3, 3, 1, 2),
    ('fs 64ch 3x3 @256', 3, 64, 64, 256, 256, 3, 3, 1, 1),
    ('fs 128->64 3x3 @256', 3, 128, 64, 256, 256, 3, 3, 1, 1),
]


def bench(fn, it=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it


def main():
    torch.manual_seed(0)
    print('%-42s %9s %9s %8s %8s %6s' % ('shape', 'v1 ms', 'rw ms', 'v1 TF/s', 'rw TF/s', 'x'))
    for name, B, cin, cout, H, W, kh, kw, s, p in SHAPES:
        x = torch.randn(B, cin, H, W, device='cuda').to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(cout, cin, kh, kw, device='cuda') * 0.05).to(torch.bfloat16).contiguous(
            memory_format=CL)
        b = torch.randn(cout, device='cuda')
        ho = (H + 2 * p - kh) // s + 1
        wo = (W + 2 * p - kw) // s + 1
        fl = 2.0 * B * ho * wo * cout * cin * kh * kw
        res = {}
        for ver in ('1', '6'):
            if ver == '1' and cin == 32:
                # v1 needs Cin % 64: the zero-padded operands the framework used to build
                xp = torch.zeros(B, 64, H, W, device='cuda', dtype=torch.bfloat16).contiguous(
                    memory_format=CL)
                xp[:, :32] = x
                wp = torch.zeros(cout, 64, kh, kw, device='cuda', dtype=torch.bfloat16).contiguous(
                    memory_format=CL)
                wp[:, :32] = w
                args = (xp, wp)
            else:
                args = (x, w)
            os.environ['IMAGINAIRE_AMD_CONV_V'] = ver
            try:
                res[ver] = bench(lambda: X.conv2d_mfma(args[0], args[1], b, s, s, p, p, 1, 1, 0.2))
                var = X.conv_last_variant()
            finally:
                os.environ.pop('IMAGINAIRE_AMD_CONV_V')
            if ver == '6' and var != 6:
                res['6'] = float('nan')
        print('%-42s %9.3f %9.3f %8.0f %8.0f %6.2f' % (
            name, res['1'], res['6'], fl / res['1'] / 1e9, fl / res['6'] / 1e9,
            res['1'] / res['6']), flush=True)


if __name__ == '__main__':
    main()
