"""Locate the first non-finite tensor inside a hipGraph-replayed training iteration.

Hooks installed BEFORE the capture keep references to (a) every G / D leaf module's forward
output and gradient-of-output, (b) every spectral-norm scale backward's inputs (grad, σ, u, v)
and result. Tensors referenced this way stay allocated in the graph pool, and each replay
rewrites them, so after a replay they can be read like eager intermediates. Lists are printed
in capture order; MODE=sn keeps only the SN-backward tensors (a smaller change to the pool's
reuse pattern), MODE=all keeps everything.

    MODE=sn python scripts/probe/graph_stash_probe.py pix2pixHD
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'tests'))
from test_graph_families_gpu import _build, _fresh  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'pix2pixHD'
mode = os.environ.get('MODE', 'sn')
from imaginaire_amd.utils.cuda_graph import make_trainer_step  # noqa: E402
from imaginaire_amd.layers import spectral_norm as snmod  # noqa: E402

torch.cuda.set_device(0)
cfg, tr, batches = _build(name, None)
pname = {}
for net in (tr.net_G, tr.net_D):
    for n, p in net.named_parameters():
        pname[p.data_ptr()] = n

stash = []
active = [False]
orig_bwd = snmod._SNScale.backward


def sn_bwd(ctx, grad):
    out = orig_bwd(ctx, grad)
    if active[0]:
        weight, u, v, sigma = ctx.saved_tensors
        tag = pname.get(weight.data_ptr(), '?')
        stash.append(('sn.grad_in ' + tag, grad))
        stash.append(('sn.sigma ' + tag, sigma))
        stash.append(('sn.u ' + tag, u))
        stash.append(('sn.v ' + tag, v))
        stash.append(('sn.dW ' + tag, out[0]))
    return out


snmod._SNScale.backward = staticmethod(sn_bwd)

if mode == 'all':
    def fwd_hook(mod, inp, out):
        if active[0]:
            for o in (out if isinstance(out, (tuple, list)) else [out]):
                if torch.is_tensor(o) and o.is_floating_point():
                    stash.append(('fwd ' + mod._probe_name, o))

    def bwd_hook(mod, gin, gout):
        if active[0]:
            for g in gout:
                if torch.is_tensor(g):
                    stash.append(('grad_out ' + mod._probe_name, g))

    for tag, net in (('G', tr.net_G), ('D', tr.net_D)):
        for n, m in net.named_modules():
            if len(list(m.children())) == 0:
                m._probe_name = tag + ':' + n
                m.register_forward_hook(fwd_hook)
                m.register_full_backward_hook(bwd_hook)

step, graphed = make_trainer_step(tr, warmup=2, enabled=True)
for i in range(2):
    step(tr.start_of_iteration(_fresh(batches[i % 2]), i))
torch.cuda.synchronize()
active[0] = True
step(tr.start_of_iteration(_fresh(batches[0]), 2))  # capture + first replay
active[0] = False
torch.cuda.synchronize()
print('stashed %d tensors during capture' % len(stash), flush=True)
params = list(tr.net_G.named_parameters())


def report(tag):
    bad = [(n, tuple(t.shape)) for n, t in stash if not torch.isfinite(t).all()]
    badp = [n for n, p in params if not torch.isfinite(p).all()]
    print('%s: %d non-finite stashed tensors; first: %s' % (tag, len(bad), bad[:8]), flush=True)
    print('   non-finite G params: %d %s' % (len(badp), badp[:4]), flush=True)
    sig = [(n, float(t.reshape(-1)[0])) for n, t in stash if n.startswith('sn.sigma')]
    print('   sigmas: %s' % sig[:6], flush=True)
    return bool(bad or badp)


report('replay 0')
for it in range(4):
    graphed(tr.start_of_iteration(_fresh(batches[1]), 3 + it))
    torch.cuda.synchronize()
    if report('replay %d' % (it + 1)):
        break
