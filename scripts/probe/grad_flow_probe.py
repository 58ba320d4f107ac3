"""Where two runs of one training iteration part ways in the BACKWARD: every leaf module's output
gradient (tensor hooks, recorded in backward order with the module's name) of the HIP-bf16 run
and of the PyTorch-bf16 run (IMAGINAIRE_AMD_EAGER=1, same autocast) are compared by cosine;
the modules are listed in backward order so the first one whose gradient turns is the culprit's
neighbour. Also prints each module's output (forward) cosine.

    python scripts/probe/grad_flow_probe.py fs_vid2vid_face.yaml:2:K2 [filter-substring]
"""
import os
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import test_model_parity_gpu as P  # noqa: E402

REC = {'on': False, 'fwd': [], 'bwd': []}


def _install(net):
    for name, m in net.named_modules():
        if len(list(m.children())):
            continue

        def fwd(mod, inp, out, name=name):
            if not REC['on'] or not torch.is_tensor(out):
                return
            REC['fwd'].append((name, out.detach().float().cpu()))
            if out.requires_grad:
                out.register_hook(lambda g, name=name: REC['bwd'].append(
                    (name, g.detach().float().cpu())) if REC['on'] else None)
        m.register_forward_hook(fwd)


_orig_get_trainer = None


def run(spec, flt):
    parts = spec.split(':')
    config = parts[0]
    seq = int(parts[1]) if len(parts) > 1 and parts[1] else None
    ov = [('data.initial_few_shot_K', int(x[1:])) for x in parts[2:] if x.startswith('K')]
    import imaginaire_amd.utils.trainer as T
    orig = T.get_trainer

    def patched(*a, **k):
        tr = orig(*a, **k)
        _install(tr.net_G)
        return tr
    P.get_trainer = patched  # noqa: the test module imports it inside _iteration
    T.get_trainer = patched
    res = {}
    for tag, eager, amp in (('hip', False, 'O1'), ('torch', True, 'O1'), ('fp32', True, 'O0')):
        REC['fwd'], REC['bwd'] = [], []
        REC['on'] = True
        P._iteration(config, amp, eager, tempfile.mkdtemp(), seq_len=seq, overrides=ov)
        REC['on'] = False
        res[tag] = (list(REC['fwd']), list(REC['bwd']))
    T.get_trainer = orig

    def cos(a, b):
        if a.shape != b.shape:
            return float('nan')
        a, b = a.reshape(-1), b.reshape(-1)
        return float(torch.dot(a, b) / (a.norm() * b.norm()).clamp_min(1e-30))
    for kind, idx in (('fwd', 0), ('bwd', 1)):
        ha, ta, fa = res['hip'][idx], res['torch'][idx], res['fp32'][idx]
        print('== %s %s: %d / %d / %d records (cos vs fp32: hip, torch-bf16)' % (
            spec, kind, len(ha), len(ta), len(fa)))
        n = min(len(ha), len(ta), len(fa))
        for i in range(n):
            (na, a), (nb, b), (nf, f) = ha[i], ta[i], fa[i]
            if flt and flt not in na:
                continue
            ch, ct = cos(a, f), cos(b, f)
            mark = '  <--' if ch < ct - 0.05 else ''
            print('%5d %-66s hip %.4f torch %.4f |hip| %.3g |fp32| %.3g%s' % (
                i, na[-66:], ch, ct, float(a.norm()), float(f.norm()), mark))


if __name__ == '__main__':
    torch.cuda.set_device(0)
    run(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else '')
