"""First module whose output differs between two fresh, identically seeded trainers (D update)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def record(data):
    from imaginaire_amd.config import Config
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer
    cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', 'spade.yaml'))
    cfg.logdir = '/tmp/imaginaire_amd_determinism'
    nets = get_model_optimizer_and_scheduler(cfg, seed=7)
    tr = get_trainer(cfg, *nets, [], None)
    rec = []
    hooks = []
    for net_name, net in (('G', tr.net_G), ('D', tr.net_D)):
        for name, m in net.named_modules():
            def hook(mod, inp, out, name=net_name + ':' + name):
                if inp and torch.is_tensor(inp[0]):
                    rec.append((name + ' <in>', inp[0].detach().float().cpu().clone()))
                for pn, pv in list(mod.named_parameters(recurse=False)) + \
                        list(mod.named_buffers(recurse=False)):
                    rec.append((name + ' .' + pn, pv.detach().float().cpu().clone()))
                if torch.is_tensor(out):
                    rec.append((name, out.detach().float().cpu().clone()))
            hooks.append(m.register_forward_hook(hook))
    torch.manual_seed(11)
    d = tr.start_of_iteration({k: (v.clone() if torch.is_tensor(v) else v)
                               for k, v in data.items()}, 0)
    tr.dis_update(d)
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    return rec


def main():
    from imaginaire_amd.config import Config
    from imaginaire_amd.datasets.synthetic import DeviceBatchSource
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.deterministic = True
    cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', 'spade.yaml'))
    src = DeviceBatchSource(cfg, 2, torch.device('cuda', 0), pool=1, seed=3)
    data = src.next()
    a = record(data)
    b = record(data)
    print('recorded', len(a), len(b))
    n = 0
    for (na, ta), (nb, tb) in zip(a, b):
        if na != nb:
            print('order differs at', na, nb)
            break
        if ta.shape != tb.shape or not torch.equal(ta, tb):
            print('DIFF', na, tuple(ta.shape),
                  float((ta - tb).abs().max()) if ta.shape == tb.shape else 'shape')
            n += 1
            if n >= 12:
                break


if __name__ == '__main__':
    main()
