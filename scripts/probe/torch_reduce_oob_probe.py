"""Does a PyTorch reduction read memory outside its input tensor on this stack? Each input is
placed inside a larger buffer whose surrounding elements are NaN bit patterns; a reduction that
only reads its own elements gives the same (finite) result as on a clean copy.

    python scripts/probe/torch_reduce_oob_probe.py
"""
import torch

torch.manual_seed(0)
cl = torch.channels_last


def embedded(shape, dtype, fmt):
    """A tensor of ``shape`` / layout living in the middle of a NaN-filled buffer."""
    ref = torch.randn(shape, device='cuda').to(dtype).contiguous(memory_format=fmt)
    n = ref.numel()
    pad = 1 << 16
    buf = torch.full((n + 2 * pad,), float('nan'), device='cuda', dtype=dtype)
    t = buf[pad:pad + n].as_strided(ref.shape, ref.stride())
    t.copy_(ref)
    return t, ref.clone()


cases = [
    ('sum23 f32acc', (1, 64, 128, 128), torch.bfloat16, cl, lambda t: t.sum((2, 3), dtype=torch.float32)),
    ('sum23 f32acc', (4, 64, 32, 32), torch.bfloat16, cl, lambda t: t.sum((2, 3), dtype=torch.float32)),
    ('sum23 f32acc', (1, 16, 128, 128), torch.bfloat16, cl, lambda t: t.sum((2, 3), dtype=torch.float32)),
    ('sum023 float', (4, 8, 256, 512), torch.bfloat16, cl, lambda t: t.float().sum((0, 2, 3))),
    ('sum0 (linear bias)', (4, 256), torch.bfloat16, torch.contiguous_format, lambda t: t.sum(0)),
    ('sum0 f32', (8, 1), torch.float32, torch.contiguous_format, lambda t: t.sum(0)),
    ('mean', (4, 3, 256, 256), torch.bfloat16, cl, lambda t: t.float().mean()),
    ('var_mean23', (4, 64, 64, 64), torch.bfloat16, cl, lambda t: torch.var_mean(t.float(), (2, 3))[0]),
    ('sum23 bf16', (2, 128, 64, 64), torch.bfloat16, cl, lambda t: t.sum((2, 3))),
    ('amax', (2, 128, 64, 64), torch.bfloat16, cl, lambda t: t.amax((2, 3))),
]
bad = 0
for name, shape, dt, fmt, fn in cases:
    t, ref = embedded(shape, dt, fmt)
    a, b = fn(t), fn(ref)
    torch.cuda.synchronize()
    fin = bool(torch.isfinite(a).all())
    e = float((a.float() - b.float()).abs().max()) if fin else float('nan')
    ok = fin and e == 0.0
    bad += not ok
    print('%-20s %-20s %s  %s' % (name, shape, 'ok' if ok else 'READS OUTSIDE', e), flush=True)
print('BAD' if bad else 'OK', bad)
