"""Synthetic datasets with the exact batch contract of the reference datasets.

There is no network and no dataset on the benchmark machines, so every model
family can be trained / benchmarked on procedurally generated data whose
tensors have the shapes and value ranges the real datasets produce:

* ``images``: [-1, 1] RGB(-like) images (smooth random fields, so the
  generator has structure to learn);
* label types with ``interpolator: NEAREST`` and ``num_channels > 1``:
  one-hot maps of random Voronoi segmentations (+ the don't-care channel when
  ``use_dont_care``); other label types (edge maps, …): [0, 1] maps;
* ``key``, ``original_h_w``, ``is_flipped``; video datasets add the time axis.

``Dataset`` is a map-style dataset (CPU, like the reference). For benchmarks
``DeviceBatchSource`` keeps a pool of compact *index* maps resident in HBM and
expands one-hot labels on the GPU per step — the MI355X-native input path
(uint8 indices over PCIe instead of 185-channel fp32 one-hot maps).
"""
import math
import random
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

from imaginaire_amd.utils.data import get_crop_h_w


def _input_types(cfg_data):
    out = OrderedDict()
    for data_type in cfg_data.input_types:
        for k in data_type:
            out[k] = data_type[k]
    return out


def _crop_hw(cfg_data, is_inference=False, is_test=False):
    names = ['test'] if is_test else (['val', 'train'] if is_inference else ['train'])
    split = None
    for n in names + ['train', 'val', 'test']:
        split = getattr(cfg_data, n, None)
        if split is not None:
            break
    aug = getattr(split, 'augmentations', None)
    try:
        return get_crop_h_w(aug)
    except Exception:
        for key in ('resize_h_w',):
            if aug is not None and hasattr(aug, key):
                h, w = str(aug[key]).split(',')
                return int(h), int(w)
        side = getattr(aug, 'resize_smallest_side', 256) if aug is not None else 256
        return side, side


def voronoi_labels(h, w, num_classes, gen, num_sites=None):
    """Random Voronoi segmentation map (int64 [h, w]) with up to num_classes labels."""
    num_sites = num_sites or max(4, min(32, num_classes))
    ys = torch.randint(0, h, (num_sites,), generator=gen)
    xs = torch.randint(0, w, (num_sites,), generator=gen)
    cls = torch.randint(0, num_classes, (num_sites,), generator=gen)
    yy = torch.arange(h).view(h, 1, 1).float()
    xx = torch.arange(w).view(1, w, 1).float()
    d = (yy - ys.view(1, 1, -1).float()) ** 2 + (xx - xs.view(1, 1, -1).float()) ** 2
    return cls[d.argmin(-1)]


def smooth_field(c, h, w, gen, scale=8):
    lo = torch.rand(c, max(1, h // scale), max(1, w // scale), generator=gen) * 2 - 1
    return F.interpolate(lo[None], size=(h, w), mode='bilinear', align_corners=False)[0]


def edge_map(labels):
    e = torch.zeros_like(labels, dtype=torch.float32)
    e[:, 1:] += (labels[:, 1:] != labels[:, :-1]).float()
    e[1:, :] += (labels[1:, :] != labels[:-1, :]).float()
    return (e > 0).float()


class Dataset(torch.utils.data.Dataset):
    """Synthetic paired / unpaired / video dataset driven by ``cfg.data``."""

    def __init__(self, cfg, is_inference=False, is_test=False):
        self.cfg = cfg
        self.cfg_data = cfg.test_data if is_test else cfg.data
        self.is_inference = is_inference
        self.is_test = is_test
        self.types = _input_types(self.cfg_data)
        self.h, self.w = _crop_hw(self.cfg_data, is_inference, is_test)
        syn = getattr(self.cfg_data, 'synthetic', None)
        self.length = int(getattr(syn, 'num_samples', 64)) if syn is not None else 64
        # video datasets (paired_videos / paired_few_shot_videos contract)
        self.is_video = 'video' in str(getattr(self.cfg_data, 'type', '')) or \
            hasattr(self.cfg_data, 'num_frames_G') or \
            int(getattr(syn, 'sequence_length', 0) or 0) > 0
        self.sequence_length_max = int(getattr(syn, 'max_sequence_length', 8) or 8) \
            if syn is not None else 8
        train = getattr(self.cfg_data, 'train', None)
        self.seq_len = int(getattr(syn, 'sequence_length', 0) or 0) if syn is not None else 0
        if self.is_video and not self.seq_len:
            self.seq_len = int(getattr(train, 'initial_sequence_length', 1) or 1) \
                if not is_inference else 1
        self.sequence_length = self.seq_len
        self.few_shot = 'few_shot' in str(getattr(self.cfg_data, 'type', ''))
        self.few_shot_K = int(getattr(self.cfg_data, 'initial_few_shot_K', 1) or 1)
        self.paired = getattr(self.cfg_data, 'paired', True)
        self.input_labels = list(getattr(self.cfg_data, 'input_labels', []))
        self.input_image = list(getattr(self.cfg_data, 'input_image', ['images']))
        self.num_classes = getattr(self.cfg_data, 'num_classes', 0)
        self.sample_class_idx = None
        self.num_style_classes = int(getattr(self.cfg_data, 'num_style_classes', 0) or 0) or 1

    def __len__(self):
        return self.length

    def get_label_lengths(self):
        lengths = OrderedDict()
        for name in self.input_labels:
            t = self.types[name]
            lengths[name] = t.num_channels + (1 if getattr(t, 'use_dont_care', False) else 0)
        return lengths

    def num_inference_sequences(self):
        return max(1, self.length // max(1, self.seq_len or 1))

    def set_inference_sequence_idx(self, *args):
        self.inference_sequence_idx = args

    def set_sequence_length(self, sequence_length):
        """Frames per training sample (vid2vid curriculum); 0 = whole sequence."""
        self.sequence_length = min(int(sequence_length) or self.sequence_length_max,
                                   self.sequence_length_max)
        self.seq_len = self.sequence_length

    def set_sample_class_idx(self, class_idx):
        self.sample_class_idx = class_idx

    def _frame(self, gen):
        h, w = self.h, self.w
        out = {}
        seg = None
        for name, t in self.types.items():
            nc = t.num_channels
            interp = getattr(t, 'interpolator', 'BILINEAR')
            if name == 'unprojections':
                continue
            if name == 'flow':
                # external flow (px) + occlusion mask, wc-vid2vid fork contract
                f = smooth_field(2, h, w, gen) * 2.0
                m = (smooth_field(1, h, w, gen) + 1) / 2
                out[name] = torch.cat([f, m], 0)
            elif name in self.input_image or name.startswith('images'):
                out[name] = smooth_field(nc, h, w, gen).clamp(-1, 1)
            elif 'densepose' in name:
                # IUV map as decoded from the 8-bit PNG: U, V in [0, 1], part index I/255
                parts = voronoi_labels(h, w, 25, gen).float() / 255.0
                uv = (smooth_field(2, h, w, gen) + 1) / 2
                out[name] = torch.cat([uv, parts[None]], 0)
            elif 'instance' in name and nc == 3:
                ids = voronoi_labels(h, w, 4, gen).float() / 255.0
                out[name] = ids[None].repeat(3, 1, 1)
            elif interp == 'NEAREST' and nc > 1:
                seg = voronoi_labels(h, w, nc, gen)
                onehot = F.one_hot(seg, nc).permute(2, 0, 1).float()
                if getattr(t, 'use_dont_care', False):
                    onehot = torch.cat([onehot, torch.zeros(1, h, w)], 0)
                out[name] = onehot
            elif 'instance' in name:
                # integer instance ids (cityscapes-style: class*1000 + k)
                inst = voronoi_labels(h, w, 8, gen, num_sites=12)
                base = seg if seg is not None else torch.zeros_like(inst)
                out[name] = (base * 1000 + inst).float()[None]
            else:
                if seg is not None and nc == 1:
                    out[name] = edge_map(seg)[None]
                else:
                    out[name] = (smooth_field(nc, h, w, gen) + 1) / 2
        return out

    def __getitem__(self, index):
        gen = torch.Generator().manual_seed(1234 + int(index))
        if self.seq_len:
            frames = [self._frame(gen) for _ in range(self.seq_len)]
            sample = {k: torch.stack([f[k] for f in frames]) for k in frames[0]}
        else:
            sample = self._frame(gen)
        few_shot = None
        if self.few_shot:
            shots = [self._frame(gen) for _ in range(self.few_shot_K)]
            few_shot = {k: torch.stack([f[k] for f in shots]) for k in shots[0]}
        data = {}
        labels = [sample[n] for n in self.input_labels if n in sample]
        if labels:
            data['label'] = torch.cat(labels, dim=-3)
        for n in self.input_image:
            if n in sample:
                data['images' if n == 'images' or len(self.input_image) == 1 else n] = sample[n]
        for n, v in sample.items():
            if n not in self.input_labels and n not in self.input_image:
                data[n] = v
        if few_shot is not None:
            shot_labels = [few_shot[n] for n in self.input_labels if n in few_shot]
            if shot_labels:
                data['few_shot_label'] = torch.cat(shot_labels, dim=-3)
            data['few_shot_images'] = few_shot[self.input_image[0]]
        if not self.paired and 'images' in data and 'images_b' not in data:
            data['images_a'] = data['images']
            gen_b = torch.Generator().manual_seed(98765 + int(index))
            data['images_b'] = smooth_field(data['images'].shape[-3], self.h, self.w,
                                            gen_b).clamp(-1, 1)
        if self.num_classes:
            data['labels'] = torch.tensor(index % self.num_classes)
        if 'images_content' in data and 'images_style' in data:
            # few-shot unpaired contract (reference unpaired_few_shot_images.py):
            # integer class ids of the content and style images.
            ncls = max(1, int(getattr(self.cfg_data, 'num_style_classes', 0) or
                              getattr(getattr(self.cfg, 'dis', None), 'num_classes', 1) or 1))
            style_cls = self.sample_class_idx if self.sample_class_idx is not None else \
                (index * 7 + 3) % ncls
            data['labels_content'] = torch.tensor(index % ncls)
            data['labels_style'] = torch.tensor(style_cls % ncls)
        data['key'] = {k: ['synthetic/%06d' % index] for k in self.types}
        data['original_h_w'] = torch.tensor([self.h, self.w])
        data['is_flipped'] = False
        return data


class DeviceBatchSource(object):
    """Resident-in-HBM synthetic batch source for benchmarks (paired image models).

    Keeps ``pool`` compact uint8 label-index maps + bf16 images on the GPU and
    builds each batch's one-hot label with a device scatter — no host work,
    no PCIe traffic in the timed loop.
    """

    def __init__(self, cfg, batch_size, device, pool=16, seed=0):
        ds = Dataset(cfg)
        # bf16 batches when the trainer runs bf16 autocast on the GPU (its first use casts)
        amp = getattr(getattr(cfg, 'trainer', None), 'amp', 'O0')
        self.dtype = torch.bfloat16 if (torch.device(device).type == 'cuda' and
                                        amp in ('O1', 'O2', 'O3', 'bf16', True)) \
            else torch.float32
        self.batch_size = batch_size
        self.device = device
        self.types = ds.types
        self.input_labels = ds.input_labels
        self.h, self.w = ds.h, ds.w
        gen = torch.Generator().manual_seed(seed)
        self.index_maps, self.images, self.extra = [], [], []
        for _ in range(pool):
            fr = ds._frame(gen)
            self.images.append(fr['images'])
            idx = {}
            extra = {}
            for name in self.input_labels:
                t = self.types[name]
                if getattr(t, 'interpolator', 'BILINEAR') == 'NEAREST' and t.num_channels > 1:
                    idx[name] = fr[name].argmax(0).to(torch.int16)
                else:
                    extra[name] = fr[name]
            self.index_maps.append(idx)
            self.extra.append(extra)
        self.images = torch.stack(self.images).to(device, self.dtype).contiguous(
            memory_format=torch.channels_last)
        self.idx = {n: torch.stack([m[n] for m in self.index_maps]).to(device)
                    for n in self.index_maps[0]}
        self.ext = {n: torch.stack([m[n] for m in self.extra]).to(device, self.dtype)
                    for n in (self.extra[0] if self.extra else {})}
        self.pool = pool
        self.step = 0

    def next(self):
        sel = torch.arange(self.step, self.step + self.batch_size, device=self.device) % self.pool
        self.step += self.batch_size
        # the label is assembled in place in ONE NHWC (= channels-last) buffer of the compute
        # dtype: one-hot channels by a scatter into their slice, dense channels copied in
        widths = []
        for name in self.input_labels:
            t = self.types[name]
            if name in self.idx:
                widths.append(t.num_channels + (1 if getattr(t, 'use_dont_care', False) else 0))
            else:
                widths.append(self.ext[name].shape[1])
        label = torch.zeros(self.batch_size, self.h, self.w, sum(widths), device=self.device,
                            dtype=self.dtype)
        off = 0
        for name, nc in zip(self.input_labels, widths):
            part = label[..., off:off + nc]
            if name in self.idx:
                ind = self.idx[name].index_select(0, sel).long()
                part.scatter_(3, ind.unsqueeze(-1), 1.0)
            else:
                part.copy_(self.ext[name].index_select(0, sel).permute(0, 2, 3, 1))
            off += nc
        label = label.permute(0, 3, 1, 2)  # [B, C, H, W] view, channels-last strides
        return {'label': label, 'images': self.images.index_select(0, sel),
                'key': {'images': ['synthetic'] * self.batch_size},
                'original_h_w': torch.tensor([[self.h, self.w]] * self.batch_size)}
