"""Dotted-type registry.

The reference resolves ``cfg.gen.type`` / ``cfg.dis.type`` / ``cfg.trainer.type``
/ ``cfg.data.type`` / dataset-op strings with ``importlib.import_module``
(utils/trainer.py:61,95-96; utils/dataset.py:24; datasets/base.py:471-513).
Reference configs name modules under ``imaginaire.*``; we accept those names
unchanged and resolve them to ``imaginaire_amd.*`` so every reference YAML runs
as-is.
"""
import importlib

_ALIASES = {
    'imaginaire.': 'imaginaire_amd.',
}
# dataset types that only this framework's unit-test configs name: the synthetic paired-video
# and few-shot-video sets are the one generator in datasets/synthetic.py (it picks the layout
# from the config), so those names resolve to it instead of to modules of their own
_MODULES = {
    'imaginaire_amd.datasets.synthetic_videos': 'imaginaire_amd.datasets.synthetic',
    'imaginaire_amd.datasets.synthetic_few_shot_videos': 'imaginaire_amd.datasets.synthetic',
}


def canonical_module_name(name):
    for src, dst in _ALIASES.items():
        if name.startswith(src) and not name.startswith(dst):
            name = dst + name[len(src):]
            break
    return _MODULES.get(name, name)


def import_module(name):
    """Import a module by (possibly reference-style) dotted name."""
    return importlib.import_module(canonical_module_name(name))


def resolve(spec):
    """Resolve ``'pkg.module::function'`` or ``'pkg.module.attr'`` to an object."""
    if '::' in spec:
        mod, fn = spec.split('::')
        return getattr(import_module(mod), fn)
    mod, _, attr = spec.rpartition('.')
    return getattr(import_module(mod), attr)
