"""Where a replayed iteration and an eager one from the same state part ways: capture the
family's step (unit-test config), then run the same iteration three times from one saved state
— replay, eager, eager again — and print the loss differences and the parameters whose D / G
gradients differ most for (replay, eager) and (eager, eager).

    python scripts/probe/graph_eager_diff_probe.py munit
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'tests'))
from test_graph_families_gpu import _build, _fresh, _losses, _state  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'munit'
seq = int(sys.argv[2]) if len(sys.argv) > 2 else None
from imaginaire_amd.utils.cuda_graph import graph_routing, make_trainer_step  # noqa: E402
torch.cuda.set_device(0)
torch.use_deterministic_algorithms(True, warn_only=True)
cfg, tr, batches = _build(name, seq)
step, graphed = make_trainer_step(tr, warmup=2, enabled=True)
for i in range(3):
    torch.manual_seed(3)
    step(tr.start_of_iteration(_fresh(batches[i % 2]), i))
torch.cuda.synchronize()
state = _state(tr)
saved = [t.detach().clone() for t in state]


def grads(net):
    return {n: p.grad.detach().float().clone() for n, p in net.named_parameters()
            if p.grad is not None}


def run(mode):
    with torch.no_grad():
        for t, c in zip(state, saved):
            t.copy_(c)
    torch.cuda.synchronize()
    d = tr.start_of_iteration(_fresh(batches[1]), 3)
    torch.manual_seed(11)
    if mode == 'replay':
        graphed(d)
    else:
        with graph_routing():
            graphed.step_fn(d)
    torch.cuda.synchronize()
    from imaginaire_amd.ops import conv as _C
    rep = _C.ps_check_report()
    nb = [(i, r) for i, r in enumerate(rep) if not r[1]]
    if rep:
        print('   [%s] backward checks %d, non-finite %d: %s' % (mode, len(rep), len(nb), nb[:6]))
    return _losses(tr), grads(tr.net_D), grads(tr.net_G)


def params(net):
    return {n: p.detach().float().clone() for n, p in net.named_parameters()}


def run2(mode):
    l, gd, gg = run(mode)
    return l, gd, gg, params(tr.net_D), params(tr.net_G)


seqn = ['replay', 'replay', 'replay', 'eager', 'replay', 'eager']
res = [run2(m) for m in seqn]
ref = res[3]
for i, (m, A) in enumerate(zip(seqn, res)):
    la, lb = A[0], ref[0]
    print('== run %d (%s) vs run 3 (eager): losses max |diff| %.3g' % (
        i, m, max(abs(la[k] - lb[k]) for k in la)))
    for k in la:
        if la[k] != lb[k]:
            print('   %-28s %.8g vs %.8g' % (k, la[k], lb[k]))
    for net, ga, gb in (('D grad', A[1], ref[1]), ('G grad', A[2], ref[2]),
                        ('D param', A[3], ref[3]), ('G param', A[4], ref[4])):
        rows = []
        for n in ga:
            if n not in gb:
                rows.append((float('inf'), n + ' (missing)'))
                continue
            d = float((ga[n] - gb[n]).norm())
            if d > 0:
                rows.append((d / max(float(gb[n].norm()), 1e-30), n))
        rows.sort(reverse=True)
        print('   %s differing: %d of %d' % (net, len(rows), len(ga)))
        for r, n in rows[:5]:
            a_, b_ = ga.get(n.replace(' (missing)', '')), gb.get(n.replace(' (missing)', ''))
            print('      %.3g  %s  |a| %.4g |b| %.4g' % (
                r, n.replace('module.module.', ''), float(a_.norm()) if a_ is not None else -1,
                float(b_.norm()) if b_ is not None else -1))
