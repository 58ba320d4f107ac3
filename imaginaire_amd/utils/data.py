"""Data helpers: channel bookkeeping (reference utils/data.py:436-520) and the
paired/unpaired augmentation pipeline (utils/data.py:26-385).

The augmentor re-implements the reference's albumentations ``ReplayCompose``
semantics natively (numpy + PIL): one random draw per sample, replayed on every
image/label/keypoint target so all modalities and frames stay aligned; NEAREST
interpolation for label-like data, BILINEAR for images; ``is_flipped`` is
reported.
"""
import math
import random

import numpy as np
from PIL import Image

from imaginaire_amd.utils.distributed import master_only_print as print

IMG_EXTENSIONS = ('jpg', 'jpeg', 'png', 'ppm', 'bmp', 'pgm', 'tif', 'tiff', 'webp',
                  'JPG', 'JPEG', 'PNG', 'PPM', 'BMP', 'PGM', 'TIF', 'TIFF', 'WEBP')
VIDEO_EXTENSIONS = 'mp4'


def _input_type_items(data_cfg):
    for data_type in data_cfg.input_types:
        for k in data_type:
            yield k, data_type[k]


def get_paired_input_image_channel_number(data_cfg):
    num_channels = 0
    for k, v in _input_type_items(data_cfg):
        if k in data_cfg.input_image:
            num_channels += v.num_channels
    return num_channels


def get_paired_input_label_channel_number(data_cfg, video=False):
    num_labels = 0
    if not hasattr(data_cfg, 'input_labels'):
        return num_labels
    for k, v in _input_type_items(data_cfg):
        if k in data_cfg.input_labels:
            num_labels += v.num_channels
            if getattr(v, 'use_dont_care', False):
                num_labels += 1
    if video:
        num_time_steps = getattr(data_cfg.train, 'initial_sequence_length', None)
        num_labels *= num_time_steps
        num_labels += get_paired_input_image_channel_number(data_cfg) * (num_time_steps - 1)
    return num_labels


def get_class_number(data_cfg):
    return data_cfg.num_classes


def get_crop_h_w(augmentation):
    for k in augmentation.__dict__.keys():
        if 'crop_h_w' in k:
            crop_h, crop_w = str(augmentation[k]).split(',')
            return int(crop_h), int(crop_w)
    raise AttributeError('no *crop_h_w augmentation found')


# ----------------------------------------------------------------------------
# Augmentation (ReplayCompose-equivalent)
# ----------------------------------------------------------------------------

NEAREST = 'nearest'
BILINEAR = 'bilinear'


def _resize(img, h, w, interp):
    """Resize an HxWxC numpy array (any dtype)."""
    if img.shape[0] == h and img.shape[1] == w:
        return img
    if interp == NEAREST:
        ys = np.minimum((np.arange(h) * img.shape[0] / h).astype(np.int64), img.shape[0] - 1)
        xs = np.minimum((np.arange(w) * img.shape[1] / w).astype(np.int64), img.shape[1] - 1)
        return img[ys][:, xs]
    chans = []
    for c in range(img.shape[2]):
        ch = img[:, :, c]
        mode = 'F'
        pil = Image.fromarray(ch.astype(np.float32), mode=mode)
        pil = pil.resize((w, h), Image.BILINEAR)
        chans.append(np.asarray(pil))
    out = np.stack(chans, 2)
    if np.issubdtype(img.dtype, np.integer):
        info = np.iinfo(img.dtype)
        out = np.clip(np.round(out), info.min, info.max)
    return out.astype(img.dtype)


def _rotate(img, angle, interp):
    if angle == 0:
        return img
    chans = []
    for c in range(img.shape[2]):
        pil = Image.fromarray(img[:, :, c].astype(np.float32), mode='F')
        pil = pil.rotate(angle, resample=Image.NEAREST if interp == NEAREST else Image.BILINEAR)
        chans.append(np.asarray(pil))
    return np.stack(chans, 2).astype(img.dtype)


class Augmentor(object):
    """Builds and replays augmentation ops (reference utils/data.py:26-385)."""

    def __init__(self, aug_list, image_data_types, interpolators, keypoint_data_types):
        self.aug_list = aug_list
        self.image_data_types = image_data_types
        self.interpolators = interpolators
        self.keypoint_data_types = keypoint_data_types or []
        self.crop_h = self.crop_w = None
        self.resize_h = self.resize_w = None
        self.original_h = self.original_w = None
        self.resize_smallest_side = None
        self.max_time_step = 1
        self.ops = self._build_augmentation_ops()
        if self.crop_h is None and self.resize_smallest_side is None and self.resize_h is None:
            raise ValueError('resize_smallest_side, resize_h_w, and crop_h_w cannot all be '
                             'missing.')
        if self.resize_smallest_side is not None:
            assert self.resize_h is None, \
                'Cannot have both `resize_smallest_side` and `resize_h_w` set.'
        if self.resize_smallest_side is None and self.resize_h is None:
            self.resize_h, self.resize_w = self.crop_h, self.crop_w
        self.is_flipped = False

    def _build_augmentation_ops(self):
        ops = []
        for key, value in self.aug_list.items():
            if key == 'resize_smallest_side':
                self.resize_smallest_side = value
            elif key == 'resize_h_w':
                h, w = str(value).split(',')
                self.resize_h, self.resize_w = int(h), int(w)
            elif key == 'random_resize_h_w_aspect':
                a0, a1 = value.find('('), value.find(')')
                amin, amax = [float(v) for v in value[a0 + 1:a1].split(',')]
                h, w = [int(v) for v in value[:a0].split(',')[:2]]
                ops.append(('random_resized_crop', (h, w, amin, amax)))
                self.resize_h, self.resize_w = h, w
            elif key == 'rotate':
                ops.append(('rotate', value))
            elif key == 'random_rotate_90':
                ops.append(('rotate90', value))
            elif key == 'random_scale_limit':
                ops.append(('scale', value))
            elif key == 'random_crop_h_w':
                h, w = str(value).split(',')
                self.crop_h, self.crop_w = int(h), int(w)
                ops.append(('random_crop', (self.crop_h, self.crop_w)))
            elif key == 'center_crop_h_w':
                h, w = str(value).split(',')
                self.crop_h, self.crop_w = int(h), int(w)
                ops.append(('center_crop', (self.crop_h, self.crop_w)))
            elif key == 'horizontal_flip':
                if value:
                    ops.append(('hflip', None))
            elif key == 'max_time_step':
                self.max_time_step = value
                assert self.max_time_step >= 1, 'max_time_step has to be at least 1'
            else:
                raise ValueError('Unknown augmentation %s' % key)
        return ops

    def _get_resize_h_w(self, height, width):
        if self.resize_smallest_side is None:
            return self.resize_h, self.resize_w
        if height <= width:
            new_height = self.resize_smallest_side
            new_width = int(np.round(new_height * width / float(height)))
        else:
            new_width = self.resize_smallest_side
            new_height = int(np.round(new_width * height / float(width)))
        return new_height, new_width

    def _draw(self, h, w):
        """Draw one set of random parameters for an (h, w) image (post-resize)."""
        params = []
        for name, arg in self.ops:
            if name == 'rotate':
                params.append(('rotate', random.uniform(-arg, arg)))
            elif name == 'rotate90':
                params.append(('rotate90', random.randint(0, 3) if random.random() < 0.5 else 0))
            elif name == 'scale':
                s = random.uniform(1.0, 1.0 + arg)
                nh, nw = int(round(h * s)), int(round(w * s))
                params.append(('resize', (nh, nw)))
                h, w = nh, nw
            elif name == 'random_crop':
                ch, cw = arg
                y0 = random.randint(0, max(0, h - ch))
                x0 = random.randint(0, max(0, w - cw))
                params.append(('crop', (y0, x0, ch, cw)))
                h, w = ch, cw
            elif name == 'center_crop':
                ch, cw = arg
                params.append(('crop', ((h - ch) // 2, (w - cw) // 2, ch, cw)))
                h, w = ch, cw
            elif name == 'random_resized_crop':
                th, tw, amin, amax = arg
                ratio = math.exp(random.uniform(math.log(amin), math.log(amax)))
                cw = min(w, int(round(math.sqrt(h * w * ratio))))
                ch = min(h, int(round(math.sqrt(h * w / ratio))))
                y0 = random.randint(0, h - ch)
                x0 = random.randint(0, w - cw)
                params.append(('crop', (y0, x0, ch, cw)))
                params.append(('resize', (th, tw)))
                h, w = th, tw
            elif name == 'hflip':
                params.append(('hflip', random.random() < 0.5))
        return params

    @staticmethod
    def _apply(img, params, interp):
        for name, p in params:
            if name == 'rotate':
                img = _rotate(img, p, interp)
            elif name == 'rotate90':
                img = np.ascontiguousarray(np.rot90(img, p)) if p else img
            elif name == 'resize':
                img = _resize(img, p[0], p[1], interp)
            elif name == 'crop':
                y0, x0, ch, cw = p
                img = img[y0:y0 + ch, x0:x0 + cw]
            elif name == 'hflip':
                if p:
                    img = np.ascontiguousarray(img[:, ::-1])
        return img

    @staticmethod
    def _apply_keypoints(kp, params, h, w):
        kp = np.array(kp, dtype=np.float32, copy=True)
        for name, p in params:
            if name == 'resize':
                kp[..., 0] *= p[1] / w
                kp[..., 1] *= p[0] / h
                h, w = p
            elif name == 'crop':
                y0, x0, ch, cw = p
                kp[..., 0] -= x0
                kp[..., 1] -= y0
                h, w = ch, cw
            elif name == 'hflip' and p:
                kp[..., 0] = w - 1 - kp[..., 0]
        return kp

    def _interp_of(self, data_type):
        interp = self.interpolators.get(data_type, BILINEAR)
        if interp in (Image.NEAREST, 'NEAREST', NEAREST, 0):
            return NEAREST
        return BILINEAR

    def _perform_paired_augmentation(self, inputs):
        params = None
        ref_hw = None
        out = {}
        for data_type in inputs:
            if data_type in self.keypoint_data_types or data_type not in self.image_data_types:
                continue
            vals = inputs[data_type]
            if not isinstance(vals, list):
                vals = [vals]
            res = []
            for value in vals:
                value = np.array(value)
                if value.ndim == 2:
                    value = value[..., np.newaxis]
                h, w = value.shape[:2]
                if params is None:
                    self.original_h, self.original_w = h, w
                    self.resize_h, self.resize_w = self._get_resize_h_w(h, w)
                    ref_hw = (h, w)
                    params = [('resize', (self.resize_h, self.resize_w))] + \
                        self._draw(self.resize_h, self.resize_w)
                res.append(self._apply(value, params, self._interp_of(data_type)))
            out[data_type] = res
        for data_type in self.keypoint_data_types:
            if data_type in inputs and params is not None:
                vals = inputs[data_type]
                if not isinstance(vals, list):
                    vals = [vals]
                out[data_type] = np.array([self._apply_keypoints(v, params, *ref_hw)
                                           for v in vals])
        is_flipped = any(n == 'hflip' and p for n, p in (params or []))
        self.is_flipped = is_flipped
        return out, is_flipped

    def _perform_unpaired_augmentation(self, inputs):
        is_flipped = {}
        for data_type in list(inputs.keys()):
            assert data_type in self.image_data_types
            augmented, flipped = self._perform_paired_augmentation({data_type: inputs[data_type]})
            inputs[data_type] = augmented[data_type]
            is_flipped[data_type] = flipped
        return inputs, is_flipped

    def perform_augmentation(self, inputs, paired):
        if paired:
            return self._perform_paired_augmentation(inputs)
        return self._perform_unpaired_augmentation(inputs)


def load_from_lmdb(keys, lmdbs):
    data = {}
    for data_type in keys:
        data.setdefault(data_type, [])
        data_type_keys = keys[data_type]
        if not isinstance(data_type_keys, list):
            data_type_keys = [data_type_keys]
        for key in data_type_keys:
            data[data_type].append(lmdbs[data_type].getitem_by_path(key.encode(), data_type))
    return data


load_from_folder = load_from_lmdb
