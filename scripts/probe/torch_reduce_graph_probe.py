"""Are PyTorch's multi-block reductions replay-safe in a hipGraph on this stack? Capture a few
torch reductions of the shapes the training steps use (per-sample bias gradients of
channels-last bf16 maps, tap-split head bias gradients, full sums), replay several times with
different inputs copied into the static input, and compare every replay with the eager result.

    python scripts/probe/torch_reduce_graph_probe.py
"""
import torch

torch.manual_seed(0)
cl = torch.channels_last
cases = {
    'sum23_cl_bf16_f32': ((1, 64, 128, 128), cl, lambda t: t.sum((2, 3), dtype=torch.float32)),
    'sum023_cl_float': ((4, 8, 256, 512), cl, lambda t: t.float().sum((0, 2, 3))),
    'sum_all_f32': ((4, 64, 64, 64), cl, lambda t: t.float().sum()),
    'mean_all': ((4, 3, 256, 512), torch.contiguous_format, lambda t: t.float().mean()),
    'sum1_nchw': ((2, 64, 64, 64), torch.contiguous_format, lambda t: t.float().sum(1)),
}
bad = 0
for name, (shape, fmt, fn) in cases.items():
    x = torch.randn(shape, device='cuda').to(torch.bfloat16).contiguous(memory_format=fmt)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(2):
            fn(x)
    torch.cuda.current_stream().wait_stream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        y = fn(x)
    errs = []
    for rep in range(4):
        x.copy_(torch.randn(shape, device='cuda').to(torch.bfloat16))
        g.replay()
        torch.cuda.synchronize()
        ref = fn(x)
        e = float((y.float() - ref.float()).abs().max())
        fin = bool(torch.isfinite(y).all())
        errs.append('%s%.3g' % ('' if fin else 'NONFINITE ', e))
        bad += (not fin) or e > 1e-3 * max(1.0, float(ref.float().abs().max()))
    print('%-20s %s' % (name, ' | '.join(errs)), flush=True)
print('BAD' if bad else 'OK', bad)
