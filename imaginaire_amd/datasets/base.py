"""Dataset base class: LMDB / folder roots + the op language
(reference datasets/base.py:28-518).

Per sample: load raw entries for every data type -> ``pre_aug_ops`` ->
(paired / unpaired) replayed augmentation -> ``post_aug_ops`` ->
``full_data_post_aug_ops`` -> to tensor (+[-1, 1] normalisation) -> one-hot
expansion of index label maps -> ``full_data_ops``. Op strings:

* ``to_tensor``, ``to_numpy``, ``decode_json`` (and ``decode_pkl``, which
  only runs when ``IMAGINAIRE_AMD_ALLOW_PICKLE=1`` because it unpickles data);
* ``convert::<module>::<fn>`` — 1-argument converter;
* ``vis::<module>::<fn>`` — 9-argument renderer (resize/crop/original size,
  flip, cfg, data) turning keypoints into an image data type;
* ``<module>::<fn>`` — 3-argument full-sample transform (cfgdata,
  is_inference, data).

``imaginaire.`` module prefixes in configs resolve to ``imaginaire_amd.``.
"""
import json
import os
from collections import OrderedDict
from functools import partial
from inspect import signature

import numpy as np
import torch
import torch.utils.data as data

from imaginaire_amd.datasets.folder import FolderDataset
from imaginaire_amd.registry import import_module
from imaginaire_amd.utils.data import (IMG_EXTENSIONS, VIDEO_EXTENSIONS, Augmentor,
                                       load_from_folder, load_from_lmdb)
from imaginaire_amd.utils.distributed import master_only_print as print
from imaginaire_amd.utils.lmdb import create_metadata

NEAREST = 'NEAREST'


def _image_to_tensor(img, normalize):
    """HxW[xC] numpy (uint8 / uint16 / float) -> CxHxW float tensor in [0,1] or [-1,1]."""
    arr = np.asarray(img)
    if arr.ndim == 2:
        arr = arr[:, :, None]
    if arr.dtype == np.uint8:
        t = torch.from_numpy(np.ascontiguousarray(arr)).permute(2, 0, 1).float().div_(255.)
    elif arr.dtype == np.uint16:
        t = torch.from_numpy(arr.astype(np.float32) / 65535.).permute(2, 0, 1)
    else:
        t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float32)).permute(2, 0, 1)
    if normalize:
        t = t.sub(0.5).div_(0.5)
    return t.contiguous()


class BaseDataset(data.Dataset):
    def __init__(self, cfg, is_inference, is_test):
        super().__init__()
        self.cfg = cfg
        self.is_inference = is_inference
        self.is_test = is_test
        if self.is_test:
            self.cfgdata = self.cfg.test_data
            data_info = self.cfgdata.test
        else:
            self.cfgdata = self.cfg.data
            data_info = self.cfgdata.val if self.is_inference else self.cfgdata.train
        self.name = self.cfgdata.name
        self.lmdb_roots = data_info.roots
        self.dataset_is_lmdb = getattr(data_info, 'is_lmdb', True)
        if self.dataset_is_lmdb:
            self.load_from_dataset = load_from_lmdb
        else:
            assert hasattr(self.cfgdata, 'paired')
            self.load_from_dataset = load_from_folder
            print('Creating metadata')
            all_filenames, all_metadata = [], []
            if self.is_test:
                cfg.data_backup = cfg.data
                cfg.data = cfg.test_data
            for root in self.lmdb_roots:
                f, m = create_metadata(data_root=root, cfg=cfg, paired=self.cfgdata['paired'])
                all_filenames.append(f)
                all_metadata.append(m)
            if self.is_test:
                cfg.data = cfg.data_backup

        self.data_types, self.dataset_data_types, self.image_data_types = [], [], []
        self.normalize, self.extensions, self.interpolators, self.num_channels = {}, {}, {}, {}
        self.pre_aug_ops, self.post_aug_ops, self.use_dont_care = {}, {}, {}
        for data_type in self.cfgdata.input_types:
            name = list(data_type.keys())
            assert len(name) == 1
            name = name[0]
            info = data_type[name]
            defaults = dict(ext=None, normalize=False, interpolator=None, pre_aug_ops='None',
                            post_aug_ops='None', use_dont_care=False, computed_on_the_fly=False,
                            num_channels=None)
            for k, v in defaults.items():
                if k not in info:
                    info[k] = v
            self.data_types.append(name)
            if not info['computed_on_the_fly']:
                self.dataset_data_types.append(name)
            self.extensions[name] = info['ext']
            self.normalize[name] = info['normalize']
            self.num_channels[name] = info['num_channels']
            self.pre_aug_ops[name] = [op.strip() for op in str(info['pre_aug_ops']).split(',')]
            self.post_aug_ops[name] = [op.strip() for op in str(info['post_aug_ops']).split(',')]
            self.use_dont_care[name] = info['use_dont_care']
            self.interpolators[name] = None
            ext = info['ext']
            if ext is not None and (ext in IMG_EXTENSIONS or ext in VIDEO_EXTENSIONS or
                                    ext == 'npy'):
                self.image_data_types.append(name)
                self.interpolators[name] = info['interpolator']
        self.cfgdata.data_types = self.data_types
        self.cfgdata.use_dont_care = [self.use_dont_care[n] for n in self.data_types]
        self.cfgdata.num_channels = [self.num_channels[n] for n in self.data_types]

        self.full_data_post_aug_ops, self.full_data_ops = [], []
        if hasattr(self.cfgdata, 'full_data_ops'):
            self.full_data_ops = [op.strip() for op in self.cfgdata.full_data_ops.split(',')]
        if hasattr(self.cfgdata, 'full_data_post_aug_ops'):
            self.full_data_post_aug_ops = [
                op.strip() for op in self.cfgdata.full_data_post_aug_ops.split(',')]
        self.input_labels = list(getattr(self.cfgdata, 'input_labels', []))
        self.keypoint_data_types = list(getattr(self.cfgdata, 'keypoint_data_types', []))
        if is_test:
            aug_list = self.cfgdata.test.augmentations
        else:
            aug_list = self.cfgdata.val.augmentations if is_inference else \
                self.cfgdata.train.augmentations
        self.augmentor = Augmentor(aug_list, self.image_data_types, self.interpolators,
                                   self.keypoint_data_types)
        self.augmentable_types = self.image_data_types + self.keypoint_data_types

        self.sequence_lists = []
        self.lmdbs = {t: [] for t in self.dataset_data_types}
        self.dataset_probability = None
        self.additional_lists = []
        for idx, root in enumerate(self.lmdb_roots):
            if self.dataset_is_lmdb:
                self._add_dataset(root)
            else:
                self._add_dataset(root, filenames=all_filenames[idx],
                                  metadata=all_metadata[idx])
        self._compute_dataset_stats()
        self.mapping, self.epoch_length = self._create_mapping()

    # -- to be provided by subclasses
    def _create_mapping(self):
        raise NotImplementedError

    def _compute_dataset_stats(self):
        pass

    def __getitem__(self, index):
        raise NotImplementedError

    def __len__(self):
        return self.epoch_length

    # -- dataset roots
    def _add_dataset(self, root, filenames=None, metadata=None):
        if filenames is None:
            with open(os.path.join(root, 'all_filenames.json')) as fin:
                sequence_list = OrderedDict(json.load(fin))
        else:
            sequence_list = filenames
        self.sequence_lists.append(sequence_list)
        additional = os.path.join(root, 'all_indices.json')
        if os.path.exists(additional):
            print('Using additional list for object indices.')
            with open(additional) as fin:
                self.additional_lists.append(OrderedDict(json.load(fin)))
        for data_type in self.dataset_data_types:
            if self.dataset_is_lmdb:
                from imaginaire_amd.datasets.lmdb import LMDBDataset
                self.lmdbs[data_type].append(LMDBDataset(os.path.join(root, data_type)))
            else:
                self.lmdbs[data_type].append(FolderDataset(os.path.join(root, data_type),
                                                           metadata))

    # -- tensor conversion
    @staticmethod
    def _encode_onehot(label_map, num_labels, use_dont_care):
        label_map = label_map.clone()
        label_map[label_map < 0] = num_labels
        label_map[label_map >= num_labels] = num_labels
        out = torch.zeros(num_labels + 1, *label_map.shape[1:])
        out.scatter_(0, label_map.long(), 1.0)
        return out if use_dont_care else out[:num_labels]

    def perform_augmentation(self, data, paired):
        aug_inputs = {t: data[t] for t in self.augmentable_types}
        augmented, is_flipped = self.augmentor.perform_augmentation(aug_inputs, paired=paired)
        for t in self.augmentable_types:
            data[t] = augmented[t]
        return data, is_flipped

    def to_tensor(self, data):
        for data_type in self.image_data_types:
            imgs = data[data_type]
            for idx in range(len(imgs)):
                img = imgs[idx]
                if isinstance(img, torch.Tensor):
                    continue
                arr = np.asarray(img)
                if arr.dtype == np.uint8 and arr.ndim == 3 and arr.shape[2] == 4:
                    # fork convention: RGB+extra channel, all scaled to [0, 1]
                    arr = arr.astype(np.float32) / 255.
                imgs[idx] = _image_to_tensor(arr, self.normalize[data_type])
        return data

    def make_one_hot(self, data):
        for data_type in self.image_data_types:
            expected = self.num_channels[data_type]
            if expected is None:
                continue
            got = data[data_type][0].size(0)
            if got < expected:
                if got != 1:
                    raise ValueError('Num channels: %d. One-hot expansion can only be done if '
                                     'image has 1 channel' % got)
                assert str(self.interpolators[data_type]).upper() == NEAREST, \
                    'Cant do one-hot on image which has been resized with BILINEAR.'
                udc = self.use_dont_care.get(data_type, False)
                for idx in range(len(data[data_type])):
                    data[data_type][idx] = self._encode_onehot(
                        data[data_type][idx] * 255.0, expected, udc)
            elif got > expected:
                raise ValueError('Data type: %s, Num channels %d > Expected num channels %d' %
                                 (data_type, got, expected))
        return data

    # -- op language
    def apply_ops(self, data, op_dict, full_data=False):
        if full_data:
            for op in op_dict:
                if op == 'None':
                    continue
                fn, op_type = self.get_op(op)
                assert op_type == 'full_data'
                data = fn(data)
            return data
        if not op_dict:
            return data
        for data_type in data:
            for op in op_dict.get(data_type, []):
                if op == 'None':
                    continue
                fn, op_type = self.get_op(op)
                data[data_type] = fn(data[data_type])
                if op_type == 'vis' and data_type not in self.image_data_types:
                    # rendered keypoints become an image data type
                    self.image_data_types.append(data_type)
                elif op_type not in ('vis', 'convert', None):
                    raise NotImplementedError(op_type)
        return data

    def get_op(self, op):
        def list_to_tensor(d):
            assert isinstance(d, list)
            return torch.from_numpy(np.array(d, dtype=np.float32))

        def decode_json_list(d):
            assert isinstance(d, list)
            return [json.loads(item) for item in d]

        def decode_pkl_list(d):
            assert isinstance(d, list)
            if os.environ.get('IMAGINAIRE_AMD_ALLOW_PICKLE', '0') != '1':
                raise ValueError('decode_pkl unpickles dataset entries; set '
                                 'IMAGINAIRE_AMD_ALLOW_PICKLE=1 for trusted data only')
            import pickle
            return [pickle.loads(item) for item in d]  # noqa: S301 (explicit opt-in)

        def list_to_numpy(d):
            assert isinstance(d, list)
            return np.array(d)
        simple = {'to_tensor': list_to_tensor, 'decode_json': decode_json_list,
                  'decode_pkl': decode_pkl_list, 'to_numpy': list_to_numpy}
        if op in simple:
            return simple[op], None
        if '::' not in op:
            raise ValueError('Unknown op: %s' % op)
        parts = op.split('::')
        if len(parts) == 2:
            module, function = parts
            function = getattr(import_module(module), function)
            assert len(signature(function).parameters) == 3, \
                'Full data functions take in (cfgdata, is_inference, full_data) as input.'
            return partial(function, self.cfgdata, self.is_inference), 'full_data'
        if len(parts) == 3:
            function_type, module, function = parts
            function = getattr(import_module(module), function)
            n = len(signature(function).parameters)
            if function_type == 'vis':
                if n != 9:
                    raise ValueError('vis function type needs to take (resize_h, resize_w, '
                                     'crop_h, crop_w, original_h, original_w, is_flipped, '
                                     'cfgdata, data) as input.')
                a = self.augmentor
                return partial(function, a.resize_h, a.resize_w, a.crop_h, a.crop_w,
                               a.original_h, a.original_w, a.is_flipped, self.cfgdata), 'vis'
            if function_type == 'convert':
                if n != 1:
                    raise ValueError('convert function type needs to take (data) as input.')
                return function, 'convert'
        raise ValueError('Unknown op: %s' % op)
