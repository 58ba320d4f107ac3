"""Locate run-to-run differences: G init across two constructions, G forward repeatability."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def build():
    from imaginaire_amd.config import Config
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer
    cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', 'spade.yaml'))
    cfg.logdir = '/tmp/imaginaire_amd_determinism'
    nets = get_model_optimizer_and_scheduler(cfg, seed=7)
    return cfg, get_trainer(cfg, *nets, [], None)


def main():
    from imaginaire_amd.datasets.synthetic import DeviceBatchSource
    torch.use_deterministic_algorithms(True, warn_only=True)
    cfg, t1 = build()
    sd1 = {k: v.detach().cpu().clone() for k, v in t1.net_G.state_dict().items()}
    cfg2, t2 = build()
    sd2 = {k: v.detach().cpu().clone() for k, v in t2.net_G.state_dict().items()}
    diff = [k for k in sd1 if not torch.equal(sd1[k], sd2[k])]
    print('init G differs in %d tensors' % len(diff), diff[:6])
    src = DeviceBatchSource(cfg, 2, torch.device('cuda', 0), pool=1, seed=3)
    data = t1.start_of_iteration(src.next(), 0)
    outs = []
    for r in range(3):
        torch.manual_seed(5)
        with torch.no_grad(), t1.autocast():
            o = t1.net_G(data)
        outs.append({k: v.detach().float().cpu() for k, v in o.items() if torch.is_tensor(v)})
    for r in (1, 2):
        print('G fwd rerun %d:' % r, {k: float((outs[r][k] - outs[0][k]).abs().max())
                                      for k in outs[0]})
    t1.net_G.eval()
    outs = []
    for r in range(2):
        torch.manual_seed(5)
        with torch.no_grad(), t1.autocast():
            o = t1.net_G(data)
        outs.append({k: v.detach().float().cpu() for k, v in o.items() if torch.is_tensor(v)})
    print('G eval fwd rerun:', {k: float((outs[1][k] - outs[0][k]).abs().max()) for k in outs[0]})


if __name__ == '__main__':
    main()
