"""Find kernels that read memory they never wrote: fill the caching allocator's free blocks
with NaN (allocate many NaN tensors of assorted sizes, then free them), run ONE eager training
iteration with forward / backward hooks on every leaf module and report the first modules
whose outputs or input gradients are non-finite, and the parameters whose gradients are.
(A hipGraph replay hands such a kernel whatever its private pool last held; eager runs usually
hand it finite leftovers, so the bug only shows under capture.)

    python scripts/probe/poison_probe.py pix2pixHD [seq_len]
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'tests'))
from test_graph_families_gpu import _build, _fresh  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'pix2pixHD'
seq = int(sys.argv[2]) if len(sys.argv) > 2 else None
torch.cuda.set_device(0)
cfg, tr, batches = _build(name, seq)
from imaginaire_amd.utils.cuda_graph import make_trainer_step  # noqa: E402
step, _ = make_trainer_step(tr, enabled=False)
for i in range(2):  # warm-up (autotune, plans)
    step(tr.start_of_iteration(_fresh(batches[i % 2]), i))
torch.cuda.synchronize()

events = []


def fwd_hook(mod, inp, out):
    outs = out if isinstance(out, (tuple, list)) else [out]
    for o in outs:
        if torch.is_tensor(o) and o.is_floating_point() and not torch.isfinite(o).all():
            events.append(('fwd', mod._probe_name, tuple(o.shape)))


def bwd_hook(mod, gin, gout):
    for tag, gs in (('grad_out', gout), ('grad_in', gin)):
        for g in gs:
            if torch.is_tensor(g) and not torch.isfinite(g).all():
                events.append((tag, mod._probe_name, tuple(g.shape)))


hooks = []
for net in (tr.net_G, tr.net_D):
    for n, m in net.named_modules():
        if len(list(m.children())) == 0:
            m._probe_name = n
            hooks.append(m.register_forward_hook(fwd_hook))
            hooks.append(m.register_full_backward_hook(bwd_hook))

import contextlib  # noqa: E402
from imaginaire_amd.utils.cuda_graph import graph_routing  # noqa: E402
# IAMD_PROBE_ROUTING=1: the kernel routing of a graphed step (every conv on k10 / k11)
routing = graph_routing if os.environ.get('IAMD_PROBE_ROUTING') == '1' else contextlib.nullcontext
for trial in range(3):
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    junk = []
    for sz in [1 << k for k in range(8, 28)] * 3:  # 256 B .. 128 MiB, three of each
        junk.append(torch.full((sz // 4,), float('nan'), device='cuda'))
    del junk
    events.clear()
    with routing():
        step(tr.start_of_iteration(_fresh(batches[1]), 10 + trial))
    torch.cuda.synchronize()
    badp = [n for n, p in list(tr.net_G.named_parameters()) + list(tr.net_D.named_parameters())
            if p.grad is not None and not torch.isfinite(p.grad).all()]
    print('trial %d: %d non-finite events, first: %s' % (trial, len(events), events[:6]), flush=True)
    print('   non-finite param grads: %d %s' % (len(badp), badp[:6]), flush=True)
    if badp or events:
        break
