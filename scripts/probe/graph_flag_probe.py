"""Locate the first non-finite value INSIDE a replayed hipGraph: every leaf module gets forward
and backward hooks that, while the step is captured, record ``isfinite(t).all()`` of its
outputs / input gradients into a preallocated device flag array (the checks become part of the
graph). After a replay the flags are read back and the first modules, in execution order, whose
values were not finite are printed.

    python scripts/probe/graph_flag_probe.py fs_vid2vid_face 2
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'tests'))
from test_graph_families_gpu import _build, _fresh  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'fs_vid2vid_face'
seq = int(sys.argv[2]) if len(sys.argv) > 2 else None
from imaginaire_amd.utils.cuda_graph import make_trainer_step  # noqa: E402
torch.cuda.set_device(0)
torch.use_deterministic_algorithms(True, warn_only=True)
cfg, tr, batches = _build(name, seq)

MAXF = 1 << 16
# IAMD_PROBE_TENSOR_HOOKS=1: backward checks through tensor hooks on module outputs instead of
# module backward hooks (which insert BackwardHookFunction nodes and change the autograd graph)
TENSOR_HOOKS = os.environ.get('IAMD_PROBE_TENSOR_HOOKS', '0') == '1'
flags = torch.ones(MAXF, dtype=torch.bool, device='cuda')
labels = []          # slot -> (kind, module name, shape), in recording order
state = {'slot': 0, 'on': False}


def record(kind, mname, t):
    if not state['on'] or not torch.is_tensor(t) or not t.is_floating_point() or t.numel() == 0:
        return
    i = state['slot']
    if i >= MAXF:
        return
    state['slot'] = i + 1
    labels.append((kind, mname, tuple(t.shape)))
    flags[i:i + 1].copy_(torch.isfinite(t.detach()).all().reshape(1))


def fwd_hook(mod, inp, out):
    for o in (out if isinstance(out, (tuple, list)) else [out]):
        record('fwd', mod._probe_name, o)
        # output-gradient check as a TENSOR hook (no BackwardHookFunction node in the graph)
        if TENSOR_HOOKS and state['on'] and torch.is_tensor(o) and o.requires_grad:
            nm = mod._probe_name
            o.register_hook(lambda g, nm=nm: record('dout', nm, g))


def bwd_hook(mod, gin, gout):
    for g in gin:
        record('bwd', mod._probe_name, g)


for net, tag in ((tr.net_G, 'G'), (tr.net_D, 'D')):
    for n, m in net.named_modules():
        if len(list(m.children())) == 0:
            m._probe_name = tag + '.' + n.replace('module.module.', '')
            m.register_forward_hook(fwd_hook)
            if not TENSOR_HOOKS:
                m.register_full_backward_hook(bwd_hook)

step, graphed = make_trainer_step(tr, warmup=2, enabled=True)
for i in range(2):
    torch.manual_seed(3)
    step(tr.start_of_iteration(_fresh(batches[i % 2]), i))
torch.cuda.synchronize()
state['on'] = True  # the capture records the checks
torch.manual_seed(3)
step(tr.start_of_iteration(_fresh(batches[0]), 2))
state['on'] = False
torch.cuda.synchronize()
print('captured:', graphed.graph is not None if hasattr(graphed, 'graph') else '?',
      '| recorded checks:', state['slot'])
for rep in range(2):
    flags.fill_(True)
    torch.manual_seed(11)
    graphed(tr.start_of_iteration(_fresh(batches[1]), 3 + rep))
    torch.cuda.synchronize()
    f = flags[:state['slot']].cpu()
    bad = [i for i in range(state['slot']) if not bool(f[i])]
    print('replay %d: %d non-finite checks' % (rep, len(bad)))
    badp = [n for n, q in tr.net_G.named_parameters()
            if not torch.isfinite(q).all() or (q.grad is not None and not torch.isfinite(q.grad).all())]
    print('   non-finite G params / grads: %d %s' % (len(badp), badp[:3]))
    for i in bad[:25]:
        print('   #%d %s %s %s' % ((i,) + labels[i]))
