"""Dataset pipeline on CPU: folder dataset -> native LMDB (scripts/build_lmdb.py)
-> paired / unpaired / few-shot loaders; native LMDB format round-trip."""
import json
import os
import random
import sys

import numpy as np
import pytest
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scripts'))

_ext = pytest.importorskip('imaginaire_amd._C')


TEMPLATE = """
logging_iter: 1
max_iter: 1
gen:
    type: imaginaire.generators.dummy
dis:
    type: imaginaire.discriminators.dummy
data:
    name: test
    type: {data_type}
    num_workers: 0
    paired: {paired}
{input_types}
{extra}
    train:
        roots: [{roots}]
        is_lmdb: {is_lmdb}
        batch_size: 1
        initial_sequence_length: 2
        augmentations:
            resize_h_w: 32, 48
            horizontal_flip: True
    val:
        roots: [{roots}]
        is_lmdb: {is_lmdb}
        batch_size: 1
        augmentations:
            resize_h_w: 32, 48
"""


def _write_folder(root, seqs=2, frames=4, paired=True):
    rng = np.random.RandomState(0)
    for s in range(seqs):
        for f in range(frames):
            name = 'seq%d/frame%03d' % (s, f)
            img = (rng.rand(40, 60, 3) * 255).astype(np.uint8)
            seg = rng.randint(0, 5, size=(40, 60)).astype(np.uint8)
            os.makedirs(os.path.join(root, 'images', 'seq%d' % s), exist_ok=True)
            os.makedirs(os.path.join(root, 'seg_maps', 'seq%d' % s), exist_ok=True)
            Image.fromarray(img).save(os.path.join(root, 'images', name + '.jpg'))
            Image.fromarray(seg).save(os.path.join(root, 'seg_maps', name + '.png'))


INPUT_TYPES = """    input_types:
        - images:
            ext: jpg
            num_channels: 3
            interpolator: BILINEAR
            normalize: True
        - seg_maps:
            ext: png
            num_channels: 5
            interpolator: NEAREST
            normalize: False
    input_image:
        - images
    input_labels:
        - seg_maps"""


def _load_cfg(tmp_path, body):
    from imaginaire_amd.config import Config
    p = tmp_path / 'cfg.yaml'
    p.write_text(body)
    return Config(str(p))


def test_lmdb_native_roundtrip(tmp_path):
    items = [(('k%05d' % i).encode(), os.urandom(random.Random(i).choice([5, 3000, 9000])))
             for i in range(500)]
    _ext.lmdb_write(str(tmp_path / 'db'), items, 4096)
    r = _ext.LmdbReader(str(tmp_path / 'db'))
    assert len(r) == 500
    assert all(r.get(k) == v for k, v in items)
    assert r.get(b'missing') is None
    assert r.keys() == sorted(k for k, _ in items)


@pytest.mark.parametrize('is_lmdb', [True, False])
def test_paired_images_and_videos(tmp_path, is_lmdb):
    src = tmp_path / 'folder'
    _write_folder(str(src))
    body = TEMPLATE
    if is_lmdb:
        import build_lmdb
        body_build = body.format(data_type='imaginaire.datasets.paired_images', roots=src,
                                 paired=True, input_types=INPUT_TYPES, extra='',
                                 is_lmdb=True)
        (tmp_path / 'b.yaml').write_text(body_build)
        build_lmdb.main(['--config', str(tmp_path / 'b.yaml'), '--data_root', str(src),
                         '--output_root', str(tmp_path / 'lmdb'), '--paired'])
        root = tmp_path / 'lmdb'
        assert json.load(open(root / 'metadata.json')) == {'images': 'jpg', 'seg_maps': 'png'}
    else:
        root = src
    for dtype, is_video in (('imaginaire.datasets.paired_images', False),
                            ('imaginaire.datasets.paired_videos', True)):
        cfg = _load_cfg(tmp_path, body.format(data_type=dtype, roots=root, paired=True,
                                              input_types=INPUT_TYPES, extra='',
                                              is_lmdb=is_lmdb))
        from imaginaire_amd.registry import import_module
        ds = import_module(dtype).Dataset(cfg, is_inference=False)
        d = ds[0]
        if is_video:
            assert d['images'].shape == (2, 3, 32, 48)
            assert d['label'].shape == (2, 5, 32, 48)
        else:
            assert d['images'].shape == (3, 32, 48)
            assert d['label'].shape == (5, 32, 48)
            assert torch.allclose(d['label'].sum(0), torch.ones(32, 48))
        assert d['images'].min() >= -1 and d['images'].max() <= 1


def test_unpaired_images_from_folder(tmp_path):
    src = tmp_path / 'folder'
    _write_folder(str(src))
    types = """    input_types:
        - images:
            ext: jpg
            num_channels: 3
            interpolator: BILINEAR
            normalize: True"""
    cfg = _load_cfg(tmp_path, TEMPLATE.format(
        data_type='imaginaire.datasets.unpaired_images', roots=src, paired=False,
        input_types=types, extra='', is_lmdb=False))
    from imaginaire_amd.datasets.unpaired_images import Dataset
    ds = Dataset(cfg, is_inference=True)
    assert len(ds) == 8
    assert ds[3]['images'].shape == (3, 32, 48)


def test_is_dense_mirror():
    import torch
    from imaginaire_amd.ops._ext import is_dense
    a = torch.randn(2, 3, 4, 5)
    assert is_dense(a) and is_dense(a.contiguous(memory_format=torch.channels_last))
    assert is_dense(torch.nn.Parameter(a)) and is_dense(a.permute(3, 1, 0, 2))
    assert not is_dense(a[:, :2]) and not is_dense(a[..., ::2])


def test_model_average_buffers_follow_module_device():
    """Every ModelAverage buffer lives on the wrapped module's device (DDP broadcasts them)."""
    import torch
    from imaginaire_amd.utils.model_average import ModelAverage
    net = torch.nn.Sequential(torch.nn.Linear(3, 3)).to('meta')
    ma = ModelAverage(net, 0.9, 0, remove_sn=False)
    assert all(b.device.type == 'meta' for b in ma.buffers())


def test_few_shot_native_videos_mjpeg_folder(tmp_path):
    """paired_few_shot_videos_native over Motion-JPEG mp4 clips (decoded by datasets/mp4.py):
    two frames of one clip become the driving / source images."""
    from imaginaire_amd.datasets.mp4 import write_mjpeg_mp4
    src = tmp_path / 'folder'
    rng = np.random.RandomState(0)
    for s in range(2):
        os.makedirs(src / 'videos' / ('seq%d' % s))
        frames = (rng.rand(6, 40, 60, 3) * 255).astype(np.uint8)
        (src / 'videos' / ('seq%d' % s) / 'clip000.mp4').write_bytes(write_mjpeg_mp4(frames))
    types = """    input_types:
        - videos:
            ext: mp4
            num_channels: 3
            interpolator: BILINEAR
            normalize: True
    input_image:
        - videos
    input_labels: []"""
    cfg = _load_cfg(tmp_path, TEMPLATE.format(
        data_type='imaginaire.datasets.paired_few_shot_videos_native', roots=src, paired=True,
        input_types=types, extra='', is_lmdb=False))
    from imaginaire_amd.datasets.paired_few_shot_videos_native import Dataset
    ds = Dataset(cfg, is_inference=False)
    d = ds[0]
    assert d['driving_images'].shape == (3, 32, 48)
    assert d['source_images'].shape == (3, 32, 48)
    assert d['driving_images'].std() > 0.1  # decoded frames, not the blank fallback
