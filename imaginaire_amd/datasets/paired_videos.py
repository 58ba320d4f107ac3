"""Paired video dataset (reference datasets/paired_videos.py:17-305): samples
``sequence_length`` frames (random temporal stride up to the augmentor's
``max_time_step``) from sequences long enough, applies the op pipeline and
one shared augmentation draw, and returns [T, C, H, W] tensors + ``label``."""
import copy
import random
from collections import OrderedDict

import torch

from imaginaire_amd.datasets.base import BaseDataset
from imaginaire_amd.model_utils.fs_vid2vid import select_object
from imaginaire_amd.utils.distributed import master_only_print as print


class Dataset(BaseDataset):
    def __init__(self, cfg, is_inference=False, sequence_length=None, is_test=False):
        if sequence_length is None:
            sequence_length = 2 if is_inference else cfg.data.train.initial_sequence_length
        self.sequence_length = sequence_length
        super().__init__(cfg, is_inference, is_test)
        self.set_sequence_length(self.sequence_length)
        self.is_video_dataset = True

    def get_label_lengths(self):
        return OrderedDict((t, self.num_channels[t]) for t in self.input_labels)

    def num_inference_sequences(self):
        assert self.is_inference
        return len(self.mapping)

    def set_inference_sequence_idx(self, index):
        assert self.is_inference and index < len(self.mapping)
        self.inference_sequence_idx = index
        self.epoch_length = len(self.mapping[index]['filenames'])

    def set_sequence_length(self, sequence_length):
        assert isinstance(sequence_length, int)
        if sequence_length > self.sequence_length_max:
            print('Requested sequence length (%d) > max sequence length (%d). Limiting.' % (
                sequence_length, self.sequence_length_max))
            sequence_length = self.sequence_length_max
        self.sequence_length = sequence_length
        self.mapping, self.epoch_length = self._create_mapping()
        print('Epoch length:', self.epoch_length)

    def _compute_dataset_stats(self):
        print('Num datasets:', len(self.sequence_lists))
        if self.sequence_length >= 1:
            lengths = [len(f) for seq in self.sequence_lists for f in seq.values()]
            print('Num sequences:', len(lengths))
            print('Max sequence length:', max(lengths) if lengths else 0)
            self.sequence_length_max = max(lengths) if lengths else 0

    def _create_mapping(self):
        length_to_key, num_selected, total_frames = {}, 0, 0
        for lmdb_idx, sequence_list in enumerate(self.sequence_lists):
            for sequence_name, filenames in sequence_list.items():
                if len(filenames) >= self.sequence_length:
                    total_frames += len(filenames)
                    length_to_key.setdefault(len(filenames), []).append({
                        'lmdb_root': self.lmdb_roots[lmdb_idx], 'lmdb_idx': lmdb_idx,
                        'sequence_name': sequence_name, 'filenames': filenames})
                    num_selected += 1
        self.mapping = length_to_key
        self.epoch_length = num_selected
        if not self.is_inference and self.epoch_length < self.cfgdata.train.batch_size * 8:
            self.epoch_length = total_frames
        if self.is_inference:
            self.mapping = [s for seqs in length_to_key.values() for s in seqs]
        return self.mapping, self.epoch_length

    def _sample_keys(self, index):
        if self.is_inference:
            assert index < self.epoch_length
            chosen = self.mapping[self.inference_sequence_idx]
            filenames = [chosen['filenames'][index]]
        else:
            time_step = random.randint(1, self.augmentor.max_time_step)
            required = 1 + (self.sequence_length - 1) * time_step
            if required > self.sequence_length_max:
                required, time_step = self.sequence_length, 1
            valid = [s for length, seqs in self.mapping.items() if length >= required
                     for s in seqs]
            chosen = random.choice(valid)
            start = random.randint(0, len(chosen['filenames']) - required)
            filenames = chosen['filenames'][start:start + required:time_step]
            assert len(filenames) == self.sequence_length
        key = copy.deepcopy(chosen)
        key['filenames'] = filenames
        return key

    @staticmethod
    def _create_sequence_keys(sequence_name, filenames):
        assert isinstance(filenames, list), 'Filenames should be a list.'
        if sequence_name.endswith('___') and sequence_name[-9:-6] == '___':
            sequence_name = sequence_name[:-9]
        return ['%s/%s' % (sequence_name, f) for f in filenames]

    def _getitem(self, index, concat=True):
        keys = self._sample_keys(index)
        lmdb_idx = keys['lmdb_idx']
        keys, lmdbs = {t: self._create_sequence_keys(keys['sequence_name'], keys['filenames'])
                       for t in self.dataset_data_types}, \
            {t: self.lmdbs[t][lmdb_idx] for t in self.dataset_data_types}
        data = self.load_from_dataset(keys, lmdbs)
        data = self.apply_ops(data, self.pre_aug_ops)
        data = select_object(data, obj_indices=None)
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
            if not self.is_video_dataset:
                data['label'] = data['label'].squeeze(0)
        if not self.is_video_dataset:
            for t in self.image_data_types:
                if t in data:
                    data[t] = data[t].squeeze(0)
        data.update(kp_data)
        data['is_flipped'] = is_flipped
        data['key'] = keys
        data['original_h_w'] = torch.IntTensor([self.augmentor.original_h,
                                                self.augmentor.original_w])
        return self.apply_ops(data, self.full_data_ops, full_data=True)

    def __getitem__(self, index):
        return self._getitem(index, concat=True)
