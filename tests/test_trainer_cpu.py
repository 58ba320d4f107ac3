"""End-to-end SPADE training steps, checkpoint round-trip and EMA semantics on CPU."""
import os

import torch

from imaginaire_amd.config import Config
from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer
from imaginaire_amd.utils.dataset import get_train_and_val_dataloader

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup(tmp_path, model_average=True):
    cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', 'spade.yaml'))
    cfg.logdir = str(tmp_path)
    cfg.trainer.model_average = model_average
    cfg.trainer.model_average_start_iteration = 0
    cfg.trainer.model_average_beta = 0.5
    train_loader, val_loader = get_train_and_val_dataloader(cfg)
    nets = get_model_optimizer_and_scheduler(cfg, seed=0)
    trainer = get_trainer(cfg, *nets, train_loader, val_loader)
    return cfg, trainer, train_loader


def test_spade_two_iterations_and_checkpoint(tmp_path):
    cfg, trainer, loader = _setup(tmp_path)
    data = next(iter(loader))
    data = trainer.start_of_iteration(data, 0)
    before = [p.detach().clone() for p in trainer.net_G_module.parameters()]
    trainer.dis_update(data)
    trainer.gen_update(data)
    after = list(trainer.net_G_module.parameters())
    changed = sum(int(not torch.equal(a, b)) for a, b in zip(before, after))
    assert changed > 0
    for k, v in trainer.gen_losses.items():
        assert torch.isfinite(v).all(), k
    path = trainer.save_checkpoint(0, 1)
    assert os.path.exists(path)
    with open(os.path.join(cfg.logdir, 'latest_checkpoint.txt')) as f:
        assert f.read().startswith('latest_checkpoint: epoch_00000_iteration_000000001')
    sd = torch.load(path, weights_only=True)
    assert set(sd) == {'net_G', 'net_D', 'opt_G', 'opt_D', 'sch_G', 'sch_D', 'current_epoch',
                       'current_iteration'}
    # reference key layout: module.module.* and module.averaged_model.*
    assert any(k.startswith('module.module.spade_generator') for k in sd['net_G'])
    assert any(k.startswith('module.averaged_model.') for k in sd['net_G'])
    assert 'module.num_updates_tracked' in sd['net_G']
    # averaged model has spectral norm removed (plain .weight)
    assert any(k.startswith('module.averaged_model.') and k.endswith('conv.weight')
               for k in sd['net_G'])
    # auto-resume
    cfg2, trainer2, _ = _setup(tmp_path)
    ep, it = trainer2.load_checkpoint(cfg2, '')
    assert (ep, it) == (0, 1)
    for (k, a), b in zip(trainer.net_G.state_dict().items(), trainer2.net_G.state_dict().values()):
        assert torch.equal(a, b), k


def test_ema_absorbs_spectral_norm(tmp_path):
    cfg, trainer, loader = _setup(tmp_path)
    ma = trainer.net_G.module
    ma.start_iteration = 0
    ma._host_updates = 10
    ma.beta = 0.0
    ma.update_average()
    src = ma.module.state_dict()
    tgt = ma.averaged_model.state_dict()
    for key in tgt:
        if key.endswith('weight') and key + '_orig' in src:
            w = src[key + '_orig']
            wm = w.reshape(w.shape[0], -1)
            sigma = torch.dot(src[key + '_u'], wm @ src[key + '_v'])
            assert torch.allclose(tgt[key], w / sigma, atol=1e-5, rtol=1e-4), key
            break


def test_inference_writes_images(tmp_path):
    cfg, trainer, loader = _setup(tmp_path, model_average=False)
    from imaginaire_amd.utils.dataset import get_test_dataloader
    cfg.inference_args = type(cfg.inference_args)(random_style=True)
    test_loader = get_test_dataloader(cfg)
    trainer.test(test_loader, str(tmp_path / 'out'), cfg.inference_args)
    files = []
    for r, _, fs in os.walk(str(tmp_path / 'out')):
        files += fs
    assert any(f.endswith('.jpg') for f in files)


def test_fused_adam_resumes_apex_style_state():
    """apex FusedAdam keeps the step in the param group and only exp_avg/exp_avg_sq per
    parameter (reference utils/trainer.py:271-281): such a state_dict must load and step."""
    import torch
    from imaginaire_amd.optimizers import FusedAdam
    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(5))
    q = torch.nn.Parameter(torch.randn(3))
    opt = FusedAdam([p, q], lr=0.01, betas=(0.0, 0.999))
    sd = {'state': {0: {'exp_avg': torch.ones(5) * 0.1, 'exp_avg_sq': torch.ones(5) * 0.01},
                    1: {'exp_avg': torch.ones(3) * 0.2, 'exp_avg_sq': torch.ones(3) * 0.04}},
          'param_groups': [{'lr': 0.01, 'betas': (0.0, 0.999), 'eps': 1e-8,
                            'weight_decay': 0.0, 'adam_w_mode': False, 'step': 7,
                            'params': [0, 1]}]}
    opt.load_state_dict(sd)
    p.grad = torch.ones(5)
    q.grad = None  # params[0]-independent group step
    p0 = p.detach().clone()
    opt.step()
    assert opt.param_groups[0]['step'] == 8
    # reference Adam math at step 8
    ref = torch.optim.Adam([torch.nn.Parameter(p0.clone())], lr=0.01, betas=(0.0, 0.999))
    rp = ref.param_groups[0]['params'][0]
    ref.state[rp] = {'step': torch.tensor(7.), 'exp_avg': torch.ones(5) * 0.1,
                     'exp_avg_sq': torch.ones(5) * 0.01}
    rp.grad = torch.ones(5)
    ref.step()
    assert torch.allclose(p.detach(), rp.detach(), atol=1e-6)
    assert 'step' not in opt.state[p]
