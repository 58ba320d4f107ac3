"""Drop-in compatibility: every project / unit-test YAML of the reference
(imaginaire.* module paths, apex AMP levels, cudnn flags, ...) loads through
this framework's Config and instantiates its generator and discriminator.
Skipped when the reference checkout is not mounted."""
import glob
import os

import pytest
import torch

REF = '/root/reference/configs'
CONFIGS = sorted(glob.glob(os.path.join(REF, '**', '*.yaml'), recursive=True))


@pytest.mark.skipif(not CONFIGS, reason='reference configs not available')
@pytest.mark.parametrize('path', CONFIGS, ids=[os.path.relpath(p, REF) for p in CONFIGS])
def test_reference_config_builds_models(path):
    from imaginaire_amd.config import Config
    from imaginaire_amd.registry import import_module
    cfg = Config(path)
    for t in (cfg.gen.type, cfg.dis.type):
        rel = t.replace('imaginaire.', '', 1).replace('.', '/') + '.py'
        if t.startswith('imaginaire.') and \
                not os.path.exists(os.path.join(os.path.dirname(REF), 'imaginaire', rel)):
            pytest.skip('%s names %s, which the reference itself does not ship' % (path, t))
    torch.manual_seed(0)
    net_G = import_module(cfg.gen.type).Generator(cfg.gen, cfg.data)
    net_D = import_module(cfg.dis.type).Discriminator(cfg.dis, cfg.data)
    assert sum(p.numel() for p in net_G.parameters()) > 0
    assert sum(p.numel() for p in net_D.parameters()) >= 0
    import_module(cfg.trainer.type)  # the trainer module resolves too
