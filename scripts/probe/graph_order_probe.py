"""Does a hipGraph replay keep the order of consecutive kernels on one stream? A chain of
(PyTorch elementwise kernel writing X_i) -> (k2 bias-gradient kernel reading X_i) pairs is
captured and replayed with fresh inputs; every replayed bias gradient is compared with the
eager result of the same inputs. A mismatch means a kernel read its input before the
producing kernel finished.

    python scripts/probe/graph_order_probe.py
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402

X = _ext.ext()
cl = torch.channels_last
torch.manual_seed(0)
shapes = [(2, 32, 128, 128), (2, 64, 64, 64), (2, 128, 32, 32), (2, 64, 16, 16)] * 40
ys = [torch.randn(s, device='cuda').to(torch.bfloat16).contiguous(memory_format=cl) for s in shapes]
gs = [torch.randn(s, device='cuda').to(torch.bfloat16).contiguous(memory_format=cl) for s in shapes]


MODE = os.environ.get('IAMD_ORDER_PRODUCER', 'kernel')


def body():
    outs = []
    for y, g in zip(ys, gs):
        if MODE == 'memcpy':  # a same-layout clone: hipMemcpyAsync device-to-device
            dx = g.clone()
        elif MODE == 'memcpy_chain':  # kernel -> memcpy -> consumer
            dx = torch.ops.aten.leaky_relu_backward(g, y, 0.2, False).clone()
        else:
            dx = torch.ops.aten.leaky_relu_backward(g, y, 0.2, False)  # torch kernel writes dx
        outs.append(X.bias_act_bwd(dx, dx, 1.0)[1])                  # k2 reads it right after
    return outs


def refresh():
    with torch.no_grad():
        for y, g in zip(ys, gs):
            y.copy_(torch.randn(y.shape, device='cuda').to(torch.bfloat16))
            g.copy_(torch.randn(g.shape, device='cuda').to(torch.bfloat16))


st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st):
    body()
    body()
torch.cuda.current_stream().wait_stream(st)
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr, stream=st):
    outs = body()
bad_total = 0
for rep in range(5):
    refresh()
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    ref = body()
    torch.cuda.synchronize()
    bad = sum(1 for a, b in zip(outs, ref) if not torch.equal(a, b))
    nonfin = sum(1 for a in outs if not torch.isfinite(a).all())
    bad_total += bad
    print('replay %d: %d of %d bias gradients differ from eager, %d non-finite' % (
        rep, bad, len(outs), nonfin), flush=True)
print('ORDER BROKEN' if bad_total else 'ORDER OK', bad_total)
