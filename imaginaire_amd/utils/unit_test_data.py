"""Synthetic *raw* datasets for the reference's end-to-end unit-test flow.

The reference's ``scripts/test_training.sh:1-90`` downloads small raw folder
datasets (``dataset/unit_test/raw/<model>``), converts them with
``scripts/build_lmdb.py`` and trains every family for ``max_iter: 2``
iterations. There is no network here, so this module writes raw folders of
the same on-disk layout procedurally from a config's ``data.input_types``:

* paired (images and videos): ``<root>/<data_type>/<sequence>/<frame>.<ext>``;
* unpaired (``images_a`` / ``images_b``): same layout, independent files;
* few-shot class datasets (``images_content`` / ``images_style``):
  ``<root>/<data_type>/<class>/<file>.<ext>`` — the class is the folder.

File contents follow the reference's conventions per data type: 8-bit RGB
photos, single-channel label-index PNGs for ``NEAREST`` multi-channel labels,
binary edge maps, 3-channel DensePose IUV maps, OpenPose JSON (``people`` with
25 body / 70 face / 2×21 hand keypoints), dlib-68 landmark JSON, and ``.npy``
flow(+mask) arrays for the fork's wc-vid2vid ``flow`` type. ``.pkl`` types are
skipped (the fork never reads unprojections, generators/wc_vid2vid.py:147).

``lmdb_config`` rewrites a config so that its train/val (and test) splits read
the built LMDBs: synthetic dataset types are replaced with the real dataset
class of the same family.
"""
import copy
import json
import math
import os
import random

import numpy as np
import yaml
from PIL import Image


def _input_types(cfgdata):
    out = []
    for item in cfgdata['input_types']:
        for name, spec in item.items():
            out.append((name, spec or {}))
    return out


def _aug_size(cfgdata):
    """(h, w) of raw images large enough for the config's augmentations."""
    aug = (cfgdata.get('train') or {}).get('augmentations') or {}

    def hw(v):
        h, w = [int(x) for x in str(v).split(',')]
        return h, w
    if 'resize_h_w' in aug:
        return hw(aug['resize_h_w'])
    for key in ('random_crop_h_w', 'center_crop_h_w'):
        if key in aug and 'resize_smallest_side' not in aug:
            return hw(aug[key])
    if 'resize_smallest_side' in aug:
        s = int(aug['resize_smallest_side'])
        return s, int(math.ceil(s * 4 / 3))
    return 256, 256


def _smooth_field(rng, h, w, ch):
    """Low-frequency random image (so resizing / cropping stays meaningful)."""
    small = rng.random((max(2, h // 32), max(2, w // 32), ch)).astype(np.float32)
    img = Image.fromarray((small * 255).astype(np.uint8).squeeze())
    img = img.resize((w, h), Image.BILINEAR)
    return np.asarray(img).reshape(h, w, ch)


def _voronoi_labels(rng, h, w, n_labels, n_seeds=12):
    ys = rng.integers(0, h, n_seeds)
    xs = rng.integers(0, w, n_seeds)
    lab = rng.integers(0, n_labels, n_seeds)
    gy, gx = np.mgrid[0:h, 0:w]
    d = (gy[None] - ys[:, None, None]) ** 2 + (gx[None] - xs[:, None, None]) ** 2
    return lab[np.argmin(d, axis=0)].astype(np.uint8 if n_labels <= 256 else np.uint16)


def _openpose(rng, h, w, n_people=1):
    def pts(n, cx, cy, spread):
        arr = []
        for _ in range(n):
            arr += [float(np.clip(cx + rng.normal(0, spread), 0, w - 1)),
                    float(np.clip(cy + rng.normal(0, spread), 0, h - 1)),
                    float(rng.uniform(0.5, 1.0))]
        return arr
    people = []
    for _ in range(n_people):
        cx, cy = rng.uniform(0.3, 0.7) * w, rng.uniform(0.3, 0.7) * h
        people.append({'pose_keypoints_2d': pts(25, cx, cy, h / 8),
                       'face_keypoints_2d': pts(70, cx, cy - h / 6, h / 40),
                       'hand_left_keypoints_2d': pts(21, cx - w / 8, cy, h / 40),
                       'hand_right_keypoints_2d': pts(21, cx + w / 8, cy, h / 40)})
    return {'version': 1.3, 'people': people}


def _dlib68(rng, h, w):
    """68 landmarks on a rough face outline (jaw, brows, nose, eyes, mouth)."""
    cx, cy, r = w / 2, h / 2, min(h, w) / 4
    pts = []
    for i in range(17):  # jaw
        a = math.pi * (1.0 + i / 16.0)
        pts.append([cx + r * math.cos(a), cy - r * math.sin(a) * 1.1])
    for i in range(10):  # brows
        pts.append([cx - r * 0.8 + i * r * 0.18, cy - r * 0.6])
    for i in range(9):  # nose bridge + base
        pts.append([cx + (i - 6) * r * 0.08 if i >= 4 else cx, cy - r * 0.4 + min(i, 4) * r * 0.12])
    for e in (-1, 1):  # eyes
        for i in range(6):
            a = 2 * math.pi * i / 6
            pts.append([cx + e * r * 0.4 + r * 0.15 * math.cos(a),
                        cy - r * 0.3 + r * 0.07 * math.sin(a)])
    for i in range(20):  # mouth
        a = 2 * math.pi * i / 20
        pts.append([cx + r * 0.35 * math.cos(a), cy + r * 0.45 + r * 0.12 * math.sin(a)])
    pts = np.asarray(pts[:68]) + rng.normal(0, 1.0, (68, 2))
    return np.clip(pts, 0, [w - 1, h - 1]).tolist()


def _write(path, name, spec, rng, h, w):
    ext = spec.get('ext', 'png')
    nc = int(spec.get('num_channels', 3) or 3)
    interp = str(spec.get('interpolator', 'BILINEAR'))
    os.makedirs(os.path.dirname(path), exist_ok=True)
    fn = path + '.' + ext
    if ext == 'json':
        obj = _dlib68(rng, h, w) if ('dlib' in name or 'landmark' in name) else _openpose(rng, h, w)
        with open(fn, 'w') as f:
            json.dump(obj, f)
    elif ext == 'npy':
        if name == 'flow' or name.startswith('flow'):
            arr = np.concatenate([rng.normal(0, 2, (h, w, 2)),
                                  (rng.random((h, w, 1)) > 0.5)], axis=2).astype(np.float32)
        else:
            arr = rng.random((h, w, nc)).astype(np.float32)
        np.save(fn, arr, allow_pickle=False)
    elif ext == 'pkl':
        return None
    elif interp == 'NEAREST' and 'densepose' in name:
        iuv = np.zeros((h, w, 3), np.uint8)
        body = _voronoi_labels(rng, h, w, 25)
        iuv[..., 2] = body  # part index (reference stores I in the last channel, BGR->RGB)
        iuv[..., 0] = rng.integers(0, 256, (h, w))
        iuv[..., 1] = rng.integers(0, 256, (h, w))
        Image.fromarray(iuv).save(fn)
    elif interp == 'NEAREST' and ('instance' in name or nc == 1):
        ids = _voronoi_labels(rng, h, w, 8).astype(np.uint8)
        img = np.repeat(ids[..., None], nc, 2) if nc == 3 else ids
        Image.fromarray(img).save(fn)
    elif interp == 'NEAREST' and nc > 1:
        lab = _voronoi_labels(rng, h, w, nc)
        Image.fromarray(lab).save(fn)
    elif nc == 1:
        edges = (rng.random((h, w)) > 0.97).astype(np.uint8) * 255
        Image.fromarray(edges).save(fn)
    else:
        img = _smooth_field(rng, h, w, 3)
        Image.fromarray(img).save(fn, quality=95) if ext in ('jpg', 'jpeg') else \
            Image.fromarray(img).save(fn)
    return fn


def _layout(cfgdata):
    names = [n for n, _ in _input_types(cfgdata)]
    if 'images_content' in names or 'images_style' in names:
        return 'few_shot_classes'
    if 'images_a' in names or 'images_b' in names:
        return 'unpaired'
    return 'paired'


def _is_video(cfgdata):
    t = str(cfgdata.get('type', ''))
    return 'video' in t or 'initial_sequence_length' in (cfgdata.get('train') or {})


def make_raw_dataset(cfg_path, root, num_sequences=2, frames_per_sequence=None, seed=0,
                     size=None):
    """Write a raw folder dataset satisfying ``cfg_path``'s ``data.input_types``.

    Returns ``(root, paired)`` — ``paired`` is the flag ``build_lmdb.py`` needs.
    """
    with open(cfg_path) as f:
        cfg = yaml.safe_load(f)
    cfgdata = cfg['data']
    rng = np.random.default_rng(seed)
    random.seed(seed)
    h, w = size or _aug_size(cfgdata)
    layout = _layout(cfgdata)
    types = [(n, s) for n, s in _input_types(cfgdata)
             if not s.get('computed_on_the_fly', False)]
    if frames_per_sequence is None:
        if _is_video(cfgdata):
            tr = cfgdata.get('train') or {}
            seq = int(tr.get('initial_sequence_length', 4) or 4)
            k = int((cfg.get('data') or {}).get('initial_few_shot_K', 1) or 1)
            frames_per_sequence = max(2 * seq, seq + k + 2, 8)
        else:
            frames_per_sequence = 2
    if layout == 'few_shot_classes':
        for name, spec in types:
            for c in range(max(2, num_sequences)):
                for i in range(frames_per_sequence):
                    _write(os.path.join(root, name, 'class%03d' % c, '%05d' % i),
                           name, spec, rng, h, w)
        return root, False
    for s in range(num_sequences):
        for i in range(frames_per_sequence):
            for name, spec in types:
                _write(os.path.join(root, name, 'seq%04d' % s, 'frame%06d' % i),
                       name, spec, rng, h, w)
    return root, layout == 'paired'


_REAL_TYPES = {
    'imaginaire.datasets.synthetic_videos': 'imaginaire.datasets.paired_videos',
    'imaginaire.datasets.synthetic_few_shot_videos': 'imaginaire.datasets.paired_few_shot_videos',
}


def _real_type(cfgdata):
    t = str(cfgdata.get('type', ''))
    if t in _REAL_TYPES:
        return _REAL_TYPES[t]
    if t.endswith('datasets.synthetic'):
        return {'few_shot_classes': 'imaginaire.datasets.unpaired_few_shot_images',
                'unpaired': 'imaginaire.datasets.unpaired_images',
                'paired': 'imaginaire.datasets.paired_images'}[_layout(cfgdata)]
    return t


def lmdb_config(cfg_path, lmdb_root, out_path, max_iter=None):
    """Write ``out_path``: ``cfg_path`` with every split reading ``lmdb_root``."""
    with open(cfg_path) as f:
        cfg = yaml.safe_load(f)
    if 'test_data' not in cfg and 'val' in cfg['data']:
        # inference reads ``test_data``: derive it from the validation split
        td = copy.deepcopy(cfg['data'])
        td['test'] = copy.deepcopy(td['val'])
        td['test']['batch_size'] = 1
        td['paired'] = _layout(td) == 'paired'
        for split in ('train', 'val'):
            td.pop(split, None)
        cfg['test_data'] = td
    for key in ('data', 'test_data'):
        d = cfg.get(key)
        if not d:
            continue
        d['type'] = _real_type(d)
        d['input_types'] = [it for it in d['input_types']
                            if all((s or {}).get('ext') != 'pkl' for s in it.values())]
        for split in ('train', 'val', 'test'):
            if split in d:
                d[split]['roots'] = [lmdb_root]
                d[split]['is_lmdb'] = True
        d.pop('synthetic', None)
    if max_iter is not None:
        cfg['max_iter'] = int(max_iter)
        cfg['snapshot_save_iter'] = int(max_iter)  # leave a checkpoint for inference tests
    with open(out_path, 'w') as f:
        yaml.safe_dump(cfg, f, sort_keys=False)
    return out_path
