"""Debug of the k10 phase-decomposed stride-2 data gradient (1x1 s2 case)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402


def run(B, cin, cout, H, W, k, s, p):
    torch.manual_seed(0)
    x = torch.randn(B, cin, H, W, device='cuda').to(torch.bfloat16)
    w = (torch.randn(cout, cin, k, k, device='cuda') / (cin * k * k) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(B, cout, Ho, Wo, device='cuda').to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ref = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), s, p)
    # python-side phases through the plain k10 forward
    dx = torch.zeros(B, cin, H, W, device='cuda')
    for ry in range(s):
        qy = (ry + p) % s
        Jy = (k - qy + s - 1) // s if qy < k else 0
        for rx in range(s):
            qx = (rx + p) % s
            Jx = (k - qx + s - 1) // s if qx < k else 0
            if Jy == 0 or Jx == 0:
                continue
            cy, cx = (ry + p - qy) // s, (rx + p - qx) // s
            wsub = w[:, :, qy::s, qx::s].flip(2, 3).transpose(0, 1).contiguous(
                memory_format=torch.channels_last)
            print('  phase', ry, rx, 'wsub', tuple(wsub.shape), wsub.stride(), flush=True)
            ay, ax = (H - ry + s - 1) // s, (W - rx + s - 1) // s
            Py, Px = Jy - 1 - cy, Jx - 1 - cx
            o = _ext.ext().conv2d_mfma(dy, wsub, None, 1, 1, Py, Px, 1, 1, 1.0).float()
            print('  phase conv out', tuple(o.shape), 'need', ay, ax, flush=True)
            dx[:, :, ry::s, rx::s] = o[:, :, :ay, :ax]
    print('python phases via k10 fwd: err %.3e' % (dx - ref).abs().max().item(), flush=True)
    got = _ext.ext().conv2d_dgrad_strided_mfma(dy, w, H, W, s, p, p).float()
    print('C++ strided: err %.3e' % (got - ref).abs().max().item(), flush=True)
    wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
    print('w', w.stride(), 'flip', w.flip(2, 3).stride(), 'wt', wt.stride(), flush=True)
    print('ref/got ch0..3 at (0,0,0):', ref[0, :4, 0, 0].tolist(), got[0, :4, 0, 0].tolist())
    print('python phases ch0..3:', dx[0, :4, 0, 0].tolist(), flush=True)


if __name__ == '__main__':
    run(2, 128, 64, 9, 14, 1, 2, 0)
    run(2, 64, 128, 15, 17, 3, 2, 1)
