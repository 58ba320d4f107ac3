"""Native TensorBoard event writer: scalars, histograms, images and the hparams plugin
(reference utils/meters.py:54-159 writes all four through torch's SummaryWriter)."""
import glob
import io
import os
import struct

import numpy as np
import torch

from imaginaire_amd.utils import tb_writer


def _only_event_file(d):
    files = glob.glob(os.path.join(d, 'events.out.tfevents.*'))
    assert len(files) == 1
    return files[0]


def test_crc32c_known_vector():
    # RFC 3720 test vector: 32 bytes of zeros
    assert tb_writer.crc32c(bytes(32)) == 0x8A9136AA


def test_scalar_roundtrip(tmp_path):
    w = tb_writer.SummaryWriter(str(tmp_path))
    for i in range(3):
        w.add_scalar('gen_update/total', 0.5 * i, i * 10)
    w.close()
    got = tb_writer.read_scalars(_only_event_file(str(tmp_path)))
    assert got == [('gen_update/total', 0.0, 0), ('gen_update/total', 0.5, 10),
                   ('gen_update/total', 1.0, 20)]


def test_image_summary_is_png(tmp_path):
    from PIL import Image
    w = tb_writer.SummaryWriter(str(tmp_path))
    img = torch.zeros(3, 8, 12)
    img[0, :4] = 1.0  # red top half
    w.add_image('Visualizations', img, 7)
    w.close()
    ev = [e for e in tb_writer.read_events(_only_event_file(str(tmp_path)))
          if e.get('kind') == 'image']
    assert len(ev) == 1
    e = ev[0]
    assert (e['tag'], e['step'], e['height'], e['width'], e['channels']) == \
        ('Visualizations', 7, 8, 12, 3)
    a = np.asarray(Image.open(io.BytesIO(e['png'])))
    assert a.shape == (8, 12, 3)
    assert (a[:4, :, 0] == 255).all() and (a[4:] == 0).all()


def test_histogram_summary(tmp_path):
    w = tb_writer.SummaryWriter(str(tmp_path))
    v = torch.arange(100, dtype=torch.float32)
    w.add_histogram('w', v, 3, bins=10)
    w.close()
    e = [e for e in tb_writer.read_events(_only_event_file(str(tmp_path)))
         if e.get('kind') == 'histogram'][0]
    assert e['tag'] == 'w' and e['step'] == 3
    assert e['min'] == 0 and e['max'] == 99 and e['num'] == 100 and e['sum'] == 4950
    assert sum(e['buckets']) == 100 and len(e['buckets']) == 10


def test_hparams_plugin_summaries(tmp_path):
    w = tb_writer.SummaryWriter(str(tmp_path))
    w.add_hparams({'lr': 1e-4, 'arch': 'spade', 'sn': True}, {'FID': 12.5})
    w.close()
    evs = tb_writer.read_events(_only_event_file(str(tmp_path)))
    plugin = [e for e in evs if e.get('kind') == 'plugin']
    assert [e['tag'] for e in plugin] == ['_hparams_/experiment',
                                          '_hparams_/session_start_info',
                                          '_hparams_/session_end_info']
    assert all(e['plugin'] == 'hparams' for e in plugin)
    # experiment lists the three hparams and the metric; session start carries the values
    exp = plugin[0]['content']
    for name in (b'lr', b'arch', b'sn', b'FID'):
        assert name in exp
    ssi = plugin[1]['content']
    assert b'spade' in ssi and struct.pack('<d', 1e-4) in ssi
    assert ('FID', 12.5, 0) in tb_writer.read_scalars(_only_event_file(str(tmp_path)))


def test_meters_route_images_and_hparams(tmp_path):
    from imaginaire_amd.utils import meters
    old = meters.LOG_WRITER
    try:
        meters.LOG_WRITER = tb_writer.SummaryWriter(str(tmp_path))
        meters.Meter('x').write_image(torch.rand(3, 4, 4), 1)
        meters.add_hparams({'a': 1}, {'m': 2.0})
        meters.LOG_WRITER.close()
        kinds = [e.get('kind') for e in tb_writer.read_events(_only_event_file(str(tmp_path)))]
        assert 'image' in kinds and kinds.count('plugin') == 3
    finally:
        meters.LOG_WRITER = old
