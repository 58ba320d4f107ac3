"""Does every kernel of a LONG replayed hipGraph see the writes of the kernel before it?

A chain of N dependent kernels over one buffer of S floats spread over the whole chip (every
kernel ``a += 1``, then one ``b = a * 2`` hop every K kernels through a second buffer and back)
is captured once and replayed; after each replay every element must equal its exact expected
value. A shortfall means a kernel read data its predecessor had not yet made visible (stale
lines in another XCD's L2, or a dispatch that did not wait for its predecessor).

    python scripts/probe/graph_coherence_probe.py [N] [S] [reps]

Round 5: the few-shot vid2vid recipe graph (~tens of thousands of nodes) read stale operands in
replays unless DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 (scripts/gpu/r5_fsnan*.sh); this probe measures
the same property on plain PyTorch kernels.
"""
import os
import sys
import time

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
size = int(sys.argv[2]) if len(sys.argv) > 2 else (1 << 22)
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
hop = 16
# MODE=kernel: the hop is two multiply kernels; MODE=copy: two device-to-device copies
# (copy_ of same-dtype contiguous tensors: memcpy nodes in the graph, not kernels)
# MODE=hip: the hop is one of the framework's HIP kernels (pad_channels_cast: a fp32 NCHW ->
# NHWC pass, every element equal so the layout change is value-preserving) and a copy back
mode = os.environ.get('MODE', 'kernel')
a = torch.zeros(size, device='cuda')
b = torch.zeros(size, device='cuda')
if mode in ('memset', 'memset4'):
    # hipMemsetAsync on the capturing stream: MEMSET graph nodes, as the few-shot vid2vid
    # graph holds (36 four-byte memsets, scripts/probe/graph_dot.py). The hop writes b, zeroes
    # it (all of it / its first 4 bytes) and adds it back to a: a memset that runs out of order
    # with its neighbours leaves a off by the b it should have cleared.
    import ctypes
    _hip = ctypes.CDLL('libamdhip64.so')
    _hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t,
                                    ctypes.c_void_p]

    def _memset(t, nbytes):
        err = _hip.hipMemsetAsync(ctypes.c_void_p(t.data_ptr()), 0, nbytes,
                                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert err == 0, err
if mode == 'hip':
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    os.environ.setdefault('IMAGINAIRE_AMD_GRAPH_ALLOW_PACKET_CAPTURE', '1')
    from imaginaire_amd.ops import _ext  # noqa: E402
    X = _ext.ext()
    a4 = a.view(1, size // 64, 8, 8)


def body():
    for i in range(n):
        if i % hop == hop - 1:
            if mode == 'copy':
                b.copy_(a)
                a.copy_(b)
            elif mode in ('memset', 'memset4'):
                torch.mul(a, 2.0, out=b)
                _memset(b, b.numel() * 4 if mode == 'memset' else 4)
                if mode == 'memset':
                    a.add_(b)
                else:
                    a[:1].add_(b[:1])
            elif mode == 'hip':
                t = X.pad_channels_cast(a4, size // 64, torch.float32)
                a4.copy_(t)
            else:
                torch.mul(a, 2.0, out=b)
                torch.mul(b, 0.5, out=a)
        else:
            a.add_(1.0)


st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st):
    body()
torch.cuda.current_stream().wait_stream(st)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
t0 = time.time()
with torch.cuda.graph(g, stream=st):
    body()
print('captured %d-op chain (%s hops) over %d floats in %.1f s (DEBUG_CLR_GRAPH_PACKET_CAPTURE=%s)' % (
    n, mode, size, time.time() - t0, os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE', 'default')),
    flush=True)
adds = sum(1 for i in range(n) if i % hop != hop - 1)
bad_total = 0
for rep in range(reps):
    a.zero_()
    torch.cuda.synchronize()
    t0 = time.time()
    g.replay()
    torch.cuda.synchronize()
    dt = time.time() - t0
    wrong = int((a != float(adds)).sum())
    bad_total += wrong
    print('replay %d: %.1f ms, %d of %d elements wrong (min %.0f, want %d)' % (
        rep, dt * 1e3, wrong, size, float(a.min()), adds), flush=True)
print('COHERENCE BROKEN' if bad_total else 'COHERENCE OK', bad_total)
