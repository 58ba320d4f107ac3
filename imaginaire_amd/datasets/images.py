"""Class-conditional image dataset (reference datasets/images.py:10-162):
the class of an image is the first path component of its sequence name."""
import random

import torch

from imaginaire_amd.datasets.base import BaseDataset


def class_mapping(dataset):
    """Per-data-type key lists annotated with class names/indices, plus the
    per-class key lists (shared by the class-conditional datasets)."""
    idx_to_key, class_names = {}, {}
    for lmdb_idx, sequence_list in enumerate(dataset.sequence_lists):
        for data_type, seqs in sequence_list.items():
            class_names.setdefault(data_type, [])
            lst = idx_to_key.setdefault(data_type, [])
            for sequence_name, filenames in seqs.items():
                class_name = sequence_name.split('/')[0]
                for filename in filenames:
                    lst.append({'lmdb_root': dataset.lmdb_roots[lmdb_idx], 'lmdb_idx': lmdb_idx,
                                'sequence_name': sequence_name, 'filename': filename,
                                'class_name': class_name})
                class_names[data_type].append(class_name)
    dataset.class_name_to_idx = {
        t: {c: i for i, c in enumerate(sorted(set(names)))} for t, names in class_names.items()}
    per_class = {}
    for t, keys in idx_to_key.items():
        per_class[t] = {i: [] for i in range(len(class_names[t]))}
        for key in keys:
            key['class_idx'] = dataset.class_name_to_idx[t][key['class_name']]
            per_class[t][key['class_idx']].append(key)
    dataset.mapping_class = per_class
    return idx_to_key, max(len(v) for v in idx_to_key.values())


def load_unpaired(dataset, per_type):
    """Shared unpaired load -> augment -> tensor pipeline for dict-of-keys samples."""
    keys, lmdbs = {}, {}
    for t in dataset.dataset_data_types:
        k = per_type[t]
        keys[t] = '%s/%s' % (k['sequence_name'], k['filename'])
        lmdbs[t] = dataset.lmdbs[t][k['lmdb_idx']]
    data = dataset.load_from_dataset(keys, lmdbs)
    data = dataset.apply_ops(data, dataset.pre_aug_ops)
    # size of the first image type before augmentation (the content image for FUNIT):
    # generators' ``keep_original_size`` inference resizes back to it
    first = next((t for t in dataset.image_data_types if t in data), None)
    orig_hw = None
    if first is not None and hasattr(data[first][0], 'shape'):
        orig_hw = tuple(int(v) for v in data[first][0].shape[:2])
    data, is_flipped = dataset.perform_augmentation(data, paired=False)
    data = dataset.apply_ops(data, dataset.post_aug_ops)
    data = dataset.apply_ops(data, dataset.full_data_post_aug_ops, full_data=True)
    data = dataset.to_tensor(data)
    for t in dataset.image_data_types:
        data[t] = data[t][0]
    data['is_flipped'] = is_flipped
    data['key'] = per_type
    if orig_hw is not None:
        data['original_h_w'] = torch.IntTensor(orig_hw)
    return data


class Dataset(BaseDataset):
    def __init__(self, cfg, is_inference=False, is_test=False):
        super().__init__(cfg, is_inference, is_test)
        self.num_classes = len(self.class_name_to_idx['images'])
        self.sample_class_idx = None

    def set_sample_class_idx(self, class_idx):
        self.sample_class_idx = class_idx
        self.epoch_length = max(len(v) for v in self.mapping.values())

    def _create_mapping(self):
        self.mapping, self.epoch_length = class_mapping(self)
        return self.mapping, self.epoch_length

    def _sample_keys(self, index):
        keys = self.mapping['images']
        return {'images': keys[index % len(keys)] if self.is_inference else random.choice(keys)}

    def __getitem__(self, index):
        per_type = self._sample_keys(index)
        data = load_unpaired(self, per_type)
        data['labels'] = per_type['images']['class_idx']
        return data
