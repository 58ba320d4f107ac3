"""Run-to-run determinism of a full SPADE training iteration on the HIP path (SURVEY §5
"deterministic kernel mode for tests").

With ``torch.use_deterministic_algorithms(True)`` every imaginaire_amd kernel on the SPADE
path reduces in a fixed order (k1 norm statistics keep one row split, k11 split-K slabs and
the spectral-norm sigma / multi-tensor norms sum per-workgroup partials in a fixed tree, k12 /
k13 gather-form backwards): two trainers built from the same seed and fed the same batch
must agree BITWISE after a D and a G update — losses, every parameter and every buffer
(BN running stats, SN u / v, EMA copy).
"""
import os

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _one_iteration(data):
    from imaginaire_amd.config import Config
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer
    cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', 'spade.yaml'))
    cfg.logdir = '/tmp/imaginaire_amd_determinism'
    cfg.trainer.model_average_start_iteration = 0
    nets = get_model_optimizer_and_scheduler(cfg, seed=7)
    trainer = get_trainer(cfg, *nets, [], None)
    torch.manual_seed(11)
    d = trainer.start_of_iteration({k: (v.clone() if torch.is_tensor(v) else v)
                                    for k, v in data.items()}, 0)
    trainer.dis_update(d)
    trainer.gen_update(d)
    torch.cuda.synchronize()
    losses = {k: v.detach().float().cpu() for k, v in trainer.gen_losses.items()}
    losses.update({'D/' + k: v.detach().float().cpu() for k, v in trainer.dis_losses.items()})
    state = {}
    for name, net in (('G', trainer.net_G), ('D', trainer.net_D)):
        for k, v in net.state_dict().items():
            state[name + '.' + k] = v.detach().cpu().clone()
    return losses, state


@pytest.mark.gpu
def test_spade_iteration_is_bitwise_reproducible():
    from imaginaire_amd.config import Config
    from imaginaire_amd.datasets.synthetic import DeviceBatchSource
    from imaginaire_amd.ops import _ext
    assert _ext.available()
    prev = torch.are_deterministic_algorithms_enabled()
    prev_cudnn = torch.backends.cudnn.deterministic
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.deterministic = True
    try:
        cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', 'spade.yaml'))
        src = DeviceBatchSource(cfg, 2, torch.device('cuda', 0), pool=1, seed=3)
        data = src.next()
        l1, s1 = _one_iteration(data)
        l2, s2 = _one_iteration(data)
    finally:
        torch.use_deterministic_algorithms(prev)
        torch.backends.cudnn.deterministic = prev_cudnn
    assert l1.keys() == l2.keys()
    for k in l1:
        assert torch.equal(l1[k], l2[k]), (k, l1[k], l2[k])
    assert s1.keys() == s2.keys()
    diff = [k for k in s1 if not torch.equal(s1[k], s2[k])]
    assert not diff, diff[:10]
