"""Few-shot paired video dataset (reference datasets/paired_few_shot_videos.py:15-315):
a driving clip plus K reference frames drawn from outside the clip of the
same sequence (or, at inference, a chosen frame of a chosen sequence).
Reference-frame tensors are returned under ``few_shot_*`` keys."""
import copy
import random

import torch

from imaginaire_amd.datasets.paired_videos import Dataset as VideoDataset
from imaginaire_amd.model_utils.fs_vid2vid import select_object
from imaginaire_amd.utils.distributed import master_only_print as print


class Dataset(VideoDataset):
    def __init__(self, cfg, is_inference=False, sequence_length=None, few_shot_K=None,
                 is_test=False):
        self.few_shot_K = cfg.data.initial_few_shot_K if few_shot_K is None else few_shot_K
        super().__init__(cfg, is_inference, sequence_length=sequence_length, is_test=is_test)

    def set_inference_sequence_idx(self, index, k_shot_index=0, k_shot_frame_index=0):
        assert self.is_inference
        assert index < len(self.mapping) and k_shot_index < len(self.mapping)
        assert k_shot_frame_index < len(self.mapping[k_shot_index]['filenames'])
        self.inference_sequence_idx = index
        self.inference_k_shot_sequence_index = k_shot_index
        self.inference_k_shot_frame_index = k_shot_frame_index
        self.epoch_length = len(self.mapping[index]['filenames'])

    def set_sequence_length(self, sequence_length, few_shot_K=None):
        few_shot_K = self.few_shot_K if few_shot_K is None else few_shot_K
        assert isinstance(sequence_length, int) and isinstance(few_shot_K, int)
        if sequence_length + few_shot_K > self.sequence_length_max:
            print('Requested sequence length (%d) + few shot K (%d) > max sequence length '
                  '(%d).' % (sequence_length, few_shot_K, self.sequence_length_max))
            sequence_length = self.sequence_length_max - few_shot_K
            print('Reduced sequence length to %s' % sequence_length)
        self.sequence_length = sequence_length
        self.few_shot_K = few_shot_K
        self.mapping, self.epoch_length = self._create_mapping()
        print('Epoch length:', self.epoch_length)

    def _create_mapping(self):
        length_to_key, num_selected = {}, 0
        has_additional = len(self.additional_lists) > 0
        for lmdb_idx, sequence_list in enumerate(self.sequence_lists):
            for sequence_name, filenames in sequence_list.items():
                if len(filenames) >= self.sequence_length + self.few_shot_K:
                    obj_indices = self.additional_lists[lmdb_idx][sequence_name] \
                        if has_additional else [0] * len(filenames)
                    length_to_key.setdefault(len(filenames), []).append({
                        'lmdb_root': self.lmdb_roots[lmdb_idx], 'lmdb_idx': lmdb_idx,
                        'sequence_name': sequence_name, 'filenames': filenames,
                        'obj_indices': obj_indices})
                    num_selected += 1
        self.mapping = length_to_key
        self.epoch_length = num_selected
        if self.is_inference:
            self.mapping = [s for seqs in length_to_key.values() for s in seqs]
        return self.mapping, self.epoch_length

    def _sample_keys(self, index):
        if self.is_inference:
            assert index < self.epoch_length
            chosen = self.mapping[self.inference_sequence_idx]
            files, objs = [chosen['filenames'][index]], [chosen['obj_indices'][index]]
            ks = self.mapping[self.inference_k_shot_sequence_index]
            fi = self.inference_k_shot_frame_index
            few_shot_key = copy.deepcopy(ks)
            few_shot_key['filenames'] = [ks['filenames'][fi]]
            few_shot_key['obj_indices'] = [ks['obj_indices'][fi]]
        else:
            time_step = random.randint(1, self.augmentor.max_time_step)
            required = 1 + (self.sequence_length - 1) * time_step
            if required + self.few_shot_K > self.sequence_length_max:
                required, time_step = self.sequence_length, 1
            valid = [s for length, seqs in self.mapping.items()
                     if length >= required + self.few_shot_K for s in seqs]
            chosen = random.choice(valid)
            n = len(chosen['filenames'])
            start = random.randint(0, n - required)
            end = start + required
            files = chosen['filenames'][start:end:time_step]
            objs = chosen['obj_indices'][start:end:time_step]
            outside = list(range(start)) + list(range(end, n))
            shots = sorted(random.sample(outside, self.few_shot_K))
            few_shot_key = copy.deepcopy(chosen)
            few_shot_key['filenames'] = [chosen['filenames'][i] for i in shots]
            few_shot_key['obj_indices'] = [chosen['obj_indices'][i] for i in shots]
            assert not set(files) & set(few_shot_key['filenames'])
            assert len(files) == self.sequence_length
        key = copy.deepcopy(chosen)
        key['filenames'], key['obj_indices'] = files, objs
        return key, few_shot_key

    def _prepare_data(self, keys, concat):
        lmdb_idx = keys['lmdb_idx']
        obj_indices = keys['obj_indices']
        seq_keys = {t: self._create_sequence_keys(keys['sequence_name'], keys['filenames'])
                    for t in self.dataset_data_types}
        lmdbs = {t: self.lmdbs[t][lmdb_idx] for t in self.dataset_data_types}
        data = self.load_from_dataset(seq_keys, lmdbs)
        data = self.apply_ops(data, self.pre_aug_ops)
        data = select_object(data, obj_indices)
        data, is_flipped = self.perform_augmentation(data, paired=True)
        kp_data = {t + '_xy': copy.deepcopy(data[t]) for t in self.keypoint_data_types}
        data = self.apply_ops(data, self.post_aug_ops)
        data = self.apply_ops(data, self.full_data_post_aug_ops, full_data=True)
        data = self.to_tensor(data)
        data = self.make_one_hot(data)
        for t in self.image_data_types:
            data[t] = torch.stack(data[t], dim=0)
        if concat and self.input_labels:
            data['label'] = torch.cat([data.pop(t) for t in self.input_labels], dim=1)
        data['is_flipped'] = is_flipped
        data['key'] = seq_keys
        data.update(kp_data)
        return data

    def _getitem(self, index, concat=True):
        keys, few_shot_keys = self._sample_keys(index)
        data = self._prepare_data(keys, concat)
        for k, v in self._prepare_data(few_shot_keys, concat).items():
            data['few_shot_' + k] = v
        if self.is_inference:
            # keep per-sequence attributes (e.g. crop boxes) identical across workers
            if 0 < index < self.cfg.data.num_workers:
                data_0 = self._getitem(0)
                if 'common_attr' in data_0:
                    self.common_attr = data['common_attr'] = data_0['common_attr']
            elif index > 0 and hasattr(self, 'common_attr'):
                data['common_attr'] = self.common_attr
        data = self.apply_ops(data, self.full_data_ops, full_data=True)
        if self.is_inference and index == 0 and 'common_attr' in data:
            self.common_attr = data['common_attr']
        return data
