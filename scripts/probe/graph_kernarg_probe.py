"""Do the kernels of a LONG linear hipGraph receive their own arguments on replay? Thousands
of tiny kernels (PyTorch fills and the k2 bias-gradient kernel), each writing a value derived
from its own arguments into its own output, are captured into one graph and replayed; every
output is checked. A mismatch means some kernel ran with another node's arguments or before
its predecessor finished.

    python scripts/probe/graph_kernarg_probe.py [n]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imaginaire_amd.ops import _ext  # noqa: E402

X = _ext.ext()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 6000
cl = torch.channels_last
outs = torch.zeros(n, 64, device='cuda')
src = [torch.full((1, 64, 8, 8), float(i % 97), device='cuda').to(torch.bfloat16).contiguous(
    memory_format=cl) for i in range(n // 2)]
res = [None] * (n // 2)


def body():
    for i in range(n // 2):
        outs[2 * i].fill_(float(i))                                   # torch fill kernel
        res[i] = X.bias_act_bwd(src[i], src[i], 1.0)[1]               # k2: 64 * (i % 97)
        outs[2 * i + 1].copy_(res[i])


st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st):
    body()
torch.cuda.current_stream().wait_stream(st)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=st):
    body()
exp = torch.zeros(n, 64, device='cuda')
for i in range(n // 2):
    exp[2 * i] = float(i)
    exp[2 * i + 1] = 64.0 * float(i % 97)
bad_total = 0
for rep in range(5):
    outs.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    bad = int((outs != exp).any(1).sum())
    bad_total += bad
    print('replay %d: %d of %d outputs wrong' % (rep, bad, n), flush=True)
print('KERNARGS BROKEN' if bad_total else 'KERNARGS OK', bad_total)
