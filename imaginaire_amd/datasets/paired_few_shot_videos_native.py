"""Few-shot dataset over native video files (reference
datasets/paired_few_shot_videos_native.py:18-226): each entry is an mp4;
two frames (random, or first/last with ``first_last_only``) become the
driving and source images.

Motion-JPEG clips are demuxed and decoded natively (``datasets/mp4.py``: ISO-BMFF sample
tables + PIL JPEG decode); other codecs (H.264 / HEVC) use the first available optional
backend (torchvision.io, imageio, PyAV) — none ships with this stack, so such clips raise an
error naming the codec.
"""
import copy
import io
import random
import tempfile
from collections import OrderedDict

import numpy as np
import torch
from PIL import Image

from imaginaire_amd.datasets import mp4
from imaginaire_amd.datasets.base import BaseDataset


def read_video_frames(buf):
    """mp4 bytes -> uint8 [T, H, W, 3] numpy array."""
    codec = None
    try:
        codec = mp4.parse_video_track(buf)['codec']
    except ValueError:
        pass  # not an ISO-BMFF file the demuxer understands: leave it to the backends
    if codec in mp4.MJPEG_CODECS:
        return mp4.decode_mjpeg_mp4(buf)
    try:
        import torchvision.io as tvio
        with tempfile.NamedTemporaryFile(suffix='.mp4') as f:
            f.write(buf)
            f.flush()
            frames, _, _ = tvio.read_video(f.name, pts_unit='sec')
        return frames.numpy()
    except ImportError:
        pass
    try:
        import imageio.v3 as iio
        return np.asarray(iio.imread(io.BytesIO(buf), index=None, extension='.mp4'))
    except ImportError:
        pass
    try:
        import av
        with av.open(io.BytesIO(buf)) as c:
            return np.stack([fr.to_ndarray(format='rgb24') for fr in c.decode(video=0)])
    except ImportError:
        raise RuntimeError('paired_few_shot_videos_native: the %s clip needs a video decoder '
                           '(torchvision.io, imageio or av; none is installed) or Motion-JPEG '
                           'encoding' % (repr(codec.decode('latin-1')) if codec else
                                         'non-mp4'))


class Dataset(BaseDataset):
    def __init__(self, cfg, is_inference=False, is_test=False):
        super().__init__(cfg, is_inference, is_test)
        self.is_video_dataset = True
        self.first_last_only = getattr(cfg.data, 'first_last_only', False)

    def get_label_lengths(self):
        return OrderedDict((t, self.num_channels[t]) for t in self.input_labels)

    def num_inference_sequences(self):
        assert self.is_inference
        return len(self.mapping)

    def _create_mapping(self):
        mapping = []
        for lmdb_idx, sequence_list in enumerate(self.sequence_lists):
            for sequence_name, filenames in sequence_list.items():
                for filename in filenames:
                    mapping.append({'lmdb_root': self.lmdb_roots[lmdb_idx],
                                    'lmdb_idx': lmdb_idx, 'sequence_name': sequence_name,
                                    'filenames': [filename]})
        self.mapping = mapping
        self.epoch_length = len(mapping)
        return self.mapping, self.epoch_length

    def _sample_keys(self, index):
        if self.is_inference:
            raise NotImplementedError('inference sampling is not defined for this dataset')
        return random.choice(self.mapping)

    @staticmethod
    def _create_sequence_keys(sequence_name, filenames):
        assert isinstance(filenames, list), 'Filenames should be a list.'
        return ['%s/%s' % (sequence_name, f) for f in filenames]

    def _getitem(self, index, concat=True):
        keys = self._sample_keys(index)
        seq_keys = {t: self._create_sequence_keys(keys['sequence_name'], keys['filenames'])
                    for t in self.dataset_data_types}
        lmdbs = {t: self.lmdbs[t][keys['lmdb_idx']] for t in self.dataset_data_types}
        data = self.load_from_dataset(seq_keys, lmdbs)
        try:
            frames = read_video_frames(data['videos'][0])
            idxs = [0, len(frames) - 1] if self.first_last_only else \
                random.sample(range(len(frames)), 2)
            data['videos'] = [Image.fromarray(frames[i]) for i in idxs]
        except (ValueError, IndexError, OSError) as e:
            print('Issue with file:', keys['sequence_name'], keys['filenames'], e)
            blank = Image.fromarray(np.zeros((512, 512, 3), dtype=np.uint8))
            data['videos'] = [blank, blank]
        data = self.apply_ops(data, self.pre_aug_ops)
        data, is_flipped = self.perform_augmentation(data, paired=True)
        kp_data = {t + '_xy': copy.deepcopy(data[t]) for t in self.keypoint_data_types}
        data = self.apply_ops(data, self.post_aug_ops)
        data = self.to_tensor(data)
        data = self.make_one_hot(data)
        for t in self.image_data_types:
            data[t] = torch.stack(data[t], dim=0)
        if concat and self.input_labels:
            data['label'] = torch.cat([data.pop(t) for t in self.input_labels], dim=1)
        data.update(kp_data)
        data['driving_images'] = data['videos'][0]
        data['source_images'] = data['videos'][1]
        data.pop('videos')
        data['is_flipped'] = is_flipped
        data['key'] = seq_keys
        data['original_h_w'] = torch.IntTensor([self.augmentor.original_h,
                                                self.augmentor.original_w])
        return self.apply_ops(data, self.full_data_ops, full_data=True)

    def __getitem__(self, index):
        return self._getitem(index, concat=True)
