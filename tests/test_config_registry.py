import os

from imaginaire_amd.config import Config, AttrDict, recursive_update, rgetattr, rsetattr
from imaginaire_amd.registry import canonical_module_name, import_module

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_config_defaults_and_yaml():
    cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', 'spade.yaml'))
    assert cfg.max_iter == 2
    assert cfg.trainer.model_average is True
    assert cfg.gen_opt.lr == 1e-4 and isinstance(cfg.gen_opt.eps, float)
    assert cfg.data.input_types[1].seg_maps.num_channels == 12
    assert cfg.trainer.gen_step == 1  # default kept
    assert rgetattr(cfg, 'gen.activation_norm_params.kernel_size') == 5
    rsetattr(cfg, 'gen.num_filters', 3)
    assert cfg.gen.num_filters == 3


def test_attrdict_roundtrip():
    d = AttrDict({'a': {'b': 1}, 'c': [{'d': 2}], 'e': 1e-4})
    assert d.a.b == 1 and d.c[0].d == 2
    y = d.yaml()
    assert y == {'a': {'b': 1}, 'c': [{'d': 2}], 'e': 1e-4}
    recursive_update(d, {'a': {'f': 3}})
    assert d.a.b == 1 and d.a.f == 3


def test_scientific_floats(tmp_path):
    p = tmp_path / 'c.yaml'
    p.write_text('gen_opt:\n  lr: 1e-4\n  eps: 1.0e-8\n')
    cfg = Config(str(p))
    assert isinstance(cfg.gen_opt.lr, float) and cfg.gen_opt.lr == 1e-4


def test_registry_aliases():
    assert canonical_module_name('imaginaire.generators.spade') == \
        'imaginaire_amd.generators.spade'
    mod = import_module('imaginaire.trainers.spade')
    assert hasattr(mod, 'Trainer')
    # the synthetic paired-video / few-shot-video types of the unit-test configs are the one
    # synthetic generator (no re-export modules of their own)
    from imaginaire_amd.datasets import synthetic
    for t in ('imaginaire.datasets.synthetic_videos',
              'imaginaire.datasets.synthetic_few_shot_videos'):
        assert canonical_module_name(t) == 'imaginaire_amd.datasets.synthetic'
        assert import_module(t).Dataset is synthetic.Dataset
