import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from imaginaire_amd.ops import _ext
ext = _ext.ext()
x = torch.zeros(4, device='cuda')
print('outside', ext.stream_capturing(), flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    f = ext.stream_capturing()
    y = x + 1
print('inside', f, flush=True)
