"""YAML configuration system.

Same schema and defaults as the reference (imaginaire/config.py:16-213): a
recursive attribute dictionary, hard defaults for every trainer / optimizer /
data knob, a YAML float resolver that accepts ``1e-4`` style literals and a
``common:`` block that is copied into both ``gen`` and ``dis``.

Differences (MI355X-first):
  * unknown keys are kept (like the reference) but ``Config.validate`` checks
    the types of the keys the framework itself reads;
  * ``trainer.amp`` accepts the apex levels ``O0/O1/O2`` and maps them to
    fp32 / bf16-autocast / bf16-params (see ``utils/amp.py``);
  * the default ``distributed_data_parallel`` is our bucketed RCCL DDP.
"""
import collections.abc
import copy
import functools
import os
import re

import yaml

from imaginaire_amd.utils.distributed import master_only_print as print

LARGE_NUMBER = 1000000000


class AttrDict(dict):
    """Dictionary whose keys are also attributes (reference config.py:16-70)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self
        for key, value in self.__dict__.items():
            self.__dict__[key] = _wrap(value)

    def yaml(self):
        out = {}
        for key, value in self.__dict__.items():
            out[key] = _unwrap(value)
        return out

    def __deepcopy__(self, memo):
        return AttrDict(copy.deepcopy(dict(self), memo))

    def __getstate__(self):
        return dict(self)

    def __setstate__(self, state):
        self.__dict__ = self
        self.update(state)

    def __repr__(self):
        lines = []
        for key, value in self.__dict__.items():
            if isinstance(value, AttrDict):
                lines.append('{}:'.format(key))
                lines += ['    ' + s for s in repr(value).split('\n')]
            elif isinstance(value, list) and value and isinstance(value[0], AttrDict):
                lines.append('{}:'.format(key))
                for item in value:
                    lines += ['    ' + s for s in repr(item).split('\n')]
            else:
                lines.append('{}: {}'.format(key, value))
        return '\n'.join(lines)


def _wrap(value):
    if isinstance(value, AttrDict):
        return value
    if isinstance(value, dict):
        return AttrDict(value)
    if isinstance(value, (list, tuple)) and len(value) > 0 and isinstance(value[0], dict):
        return [AttrDict(v) for v in value]
    return value


def _unwrap(value):
    if isinstance(value, AttrDict):
        return value.yaml()
    if isinstance(value, list):
        return [_unwrap(v) for v in value]
    return value


def _yaml_loader():
    """SafeLoader with a resolver for scientific-notation floats (reference config.py:154-164)."""
    class _Loader(yaml.SafeLoader):
        pass
    _Loader.add_implicit_resolver(
        u'tag:yaml.org,2002:float',
        re.compile(u'''^(?:
         [-+]?(?:[0-9][0-9_]*)\\.[0-9_]*(?:[eE][-+]?[0-9]+)?
        |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
        |\\.[0-9_]+(?:[eE][-+][0-9]+)?
        |[-+]?[0-9][0-9_]*(?::[0-5]?[0-9])+\\.[0-9_]*
        |[-+]?\\.(?:inf|Inf|INF)
        |\\.(?:nan|NaN|NAN))$''', re.X),
        list(u'-+0123456789.'))
    return _Loader


def load_yaml(filename):
    with open(filename, 'r') as f:
        return yaml.load(f, Loader=_yaml_loader())


class Config(AttrDict):
    """Training configuration with reference defaults (config.py:73-182)."""

    def __init__(self, filename=None, verbose=False, overrides=None):
        super().__init__()
        self.snapshot_save_iter = LARGE_NUMBER
        self.snapshot_save_epoch = LARGE_NUMBER
        self.snapshot_save_start_iter = 0
        self.snapshot_save_start_epoch = 0
        self.image_save_iter = LARGE_NUMBER
        self.image_display_iter = LARGE_NUMBER
        self.max_epoch = LARGE_NUMBER
        self.max_iter = LARGE_NUMBER
        self.logging_iter = 100
        self.trainer = AttrDict(
            model_average=False,
            model_average_beta=0.9999,
            model_average_start_iteration=1000,
            model_average_batch_norm_estimation_iteration=30,
            model_average_remove_sn=True,
            image_to_tensorboard=False,
            hparam_to_tensorboard=False,
            distributed_data_parallel='pytorch',
            delay_allreduce=True,
            gan_relativistic=False,
            gen_step=1,
            dis_step=1,
            amp='O0')
        self.gen = AttrDict(type='imaginaire.generators.dummy')
        self.dis = AttrDict(type='imaginaire.discriminators.dummy')
        for name in ('gen_opt', 'dis_opt'):
            self[name] = AttrDict(
                type='adam', fused_opt=True, lr=0.0001, adam_beta1=0.0,
                adam_beta2=0.999, eps=1e-8,
                lr_policy=AttrDict(iteration_mode=False, type='step',
                                   step_size=LARGE_NUMBER, gamma=1))
            self.__dict__[name] = self[name]
        self.data = AttrDict(name='dummy', type='imaginaire.datasets.images',
                             num_workers=0)
        self.test_data = AttrDict(name='dummy', type='imaginaire.datasets.images',
                                  num_workers=0,
                                  test=AttrDict(is_lmdb=False, roots='',
                                                batch_size=1))
        self.cudnn = AttrDict(deterministic=False, benchmark=True)
        self.pretrained_weight = ''
        self.inference_args = AttrDict()

        if filename is None:
            return
        assert os.path.exists(filename), 'File {} not exist.'.format(filename)
        cfg_dict = load_yaml(filename) or {}
        recursive_update(self, cfg_dict)
        if overrides:
            recursive_update(self, overrides)
        if 'common' in cfg_dict:
            self.common = AttrDict(**cfg_dict['common'])
            self.gen.common = self.common
            self.dis.common = self.common
        self.validate()
        if verbose:
            print(' imaginaire config '.center(80, '-'))
            print(self.__repr__())
            print(''.center(80, '-'))

    def validate(self):
        """Type-check the knobs the framework reads directly."""
        ints = ['logging_iter', 'max_iter', 'max_epoch', 'snapshot_save_iter',
                'snapshot_save_epoch', 'image_save_iter']
        for k in ints:
            v = getattr(self, k)
            if not isinstance(v, (int, float)):
                raise TypeError('config key {} must be numeric, got {!r}'.format(k, v))
        for name in ('gen_opt', 'dis_opt'):
            opt = getattr(self, name)
            if not isinstance(opt.lr, (int, float)):
                raise TypeError('{}.lr must be numeric'.format(name))
        amp = getattr(self.trainer, 'amp', 'O0')
        if amp not in ('O0', 'O1', 'O2', 'O3', 'bf16', 'fp32', False, None):
            raise ValueError('trainer.amp must be one of O0/O1/O2/O3/bf16/fp32')


def rsetattr(obj, attr, val):
    """Recursively set an attribute (reference config.py:185-188)."""
    pre, _, post = attr.rpartition('.')
    return setattr(rgetattr(obj, pre) if pre else obj, post, val)


def rgetattr(obj, attr, *args):
    """Recursively get an attribute (reference config.py:191-198)."""
    def _getattr(obj, attr):
        return getattr(obj, attr, *args)
    return functools.reduce(_getattr, [obj] + attr.split('.'))


def recursive_update(d, u):
    """Recursively merge mapping ``u`` into AttrDict ``d`` (reference config.py:201-213)."""
    for key, value in u.items():
        if isinstance(value, collections.abc.Mapping):
            d.__dict__[key] = recursive_update(d.get(key, AttrDict({})), value)
        elif isinstance(value, (list, tuple)) and len(value) > 0 \
                and isinstance(value[0], dict):
            d.__dict__[key] = [AttrDict(item) for item in value]
        else:
            d.__dict__[key] = value
    return d
