"""Does the per-sample (hyper) conv path read memory it never wrote? Record the shapes the
fs_vid2vid unit iteration sends through ``conv2d_per_sample``, then run each shape's forward
and backward standalone after filling the caching allocator's free memory with NaN, and
compare against an fp32 per-sample loop.

    python scripts/probe/per_sample_poison_probe.py
"""
import os
import sys

import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'tests'))
import test_model_parity_gpu as T  # noqa: E402
from imaginaire_amd.ops import conv as C  # noqa: E402

shapes = set()
orig = C.conv2d_per_sample


def rec(x, w, bias, padding, dilation=1):
    shapes.add((tuple(x.shape), tuple(w.shape), bias is not None, C._pair(padding),
                C._pair(dilation), x.dtype, w.dtype))
    return orig(x, w, bias, padding, dilation)


C.conv2d_per_sample = rec
T._iteration('fs_vid2vid_face.yaml', 'O1', False, '/tmp/psp', seq_len=2)
C.conv2d_per_sample = orig
print('%d per-sample shapes' % len(shapes))


def poison():
    free = torch.cuda.mem_get_info()[0]
    blobs = []
    for _ in range(8):
        try:
            blobs.append(torch.full((64 << 20,), float('nan'), device='cuda'))
        except RuntimeError:
            break
    del blobs
    torch.cuda.synchronize()
    return free


bad = 0
for xs, ws, has_b, pad, dil, xdt, wdt in sorted(shapes, key=str):
    torch.manual_seed(1)
    x = torch.randn(xs, device='cuda').to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    w = (torch.randn(ws, device='cuda') / (ws[2] * ws[3] * ws[4]) ** 0.5).to(
        torch.bfloat16).requires_grad_(True)
    b = (torch.randn(ws[0], ws[1], device='cuda') * 0.1).requires_grad_(True) if has_b else None
    poison()
    y = orig(x, w, b, pad, dil)
    g = torch.randn_like(y)
    poison()
    y.backward(g)
    torch.cuda.synchronize()
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if has_b else None
    yr = torch.stack([F.conv2d(xr[i:i + 1], wr[i], None if br is None else br[i], 1, pad,
                               dil)[0] for i in range(xs[0])])
    yr.backward(g.float())
    errs = []
    for name, got, ref in (('y', y, yr), ('dx', x.grad, xr.grad), ('dw', w.grad, wr.grad),
                           ('db', None if b is None else b.grad, None if br is None else br.grad)):
        if got is None:
            continue
        fin = bool(torch.isfinite(got).all())
        e = float((got.float() - ref).abs().max()) / max(1e-6, float(ref.abs().max()))
        errs.append('%s %s%.2g' % (name, '' if fin else 'NONFINITE ', e))
        bad += (not fin) or e > 3e-2
    print('x %-20s w %-24s b %d pad %s: %s' % (xs, ws, has_b, pad, ' | '.join(errs)), flush=True)
print('BAD' if bad else 'OK', bad)

# the same fwd + bwd captured in a hipGraph (private pool), replayed twice after poisoning
print('--- graph capture')
gbad = 0
for xs, ws, has_b, pad, dil, xdt, wdt in sorted(shapes, key=str):
    torch.manual_seed(1)
    x = torch.randn(xs, device='cuda').to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    w = (torch.randn(ws, device='cuda') / (ws[2] * ws[3] * ws[4]) ** 0.5).to(
        torch.bfloat16).requires_grad_(True)
    b = (torch.randn(ws[0], ws[1], device='cuda') * 0.1).requires_grad_(True) if has_b else None
    g = torch.randn((xs[0], ws[1]) + tuple(xs[2:]), device='cuda')
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(2):  # warm-up on the capture stream
            x.grad = w.grad = None
            if b is not None:
                b.grad = None
            orig(x, w, b, pad, dil).backward(g.to(torch.bfloat16))
    torch.cuda.current_stream().wait_stream(st)
    ref = [t.grad.detach().clone() for t in (x, w, b) if t is not None]
    x.grad = w.grad = None
    if b is not None:
        b.grad = None
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=st):
        orig(x, w, b, pad, dil).backward(g.to(torch.bfloat16))
    outs = []
    for _ in range(2):
        poison()
        gr.replay()
        torch.cuda.synchronize()
        outs.append([t.grad.detach().clone() for t in (x, w, b) if t is not None])
    msg = []
    for rep in outs:
        for name, a, r in zip(('dx', 'dw', 'db'), rep, ref):
            fin = bool(torch.isfinite(a).all())
            e = float((a.float() - r.float()).abs().max())
            msg.append('%s %s%.2g' % (name, '' if fin else 'NONFINITE ', e))
            gbad += (not fin) or e > 0
    print('x %-20s w %-24s: %s' % (xs, ws, ' | '.join(msg)), flush=True)
print('GRAPH BAD' if gbad else 'GRAPH OK', gbad)
