"""End-to-end unit training from real LMDBs (reference scripts/test_training.sh:1-90):
synthetic raw folders -> scripts/build_lmdb.py -> train.py for one iteration, one config per
dataset class (paired images, unpaired, few-shot classes, paired videos with OpenPose JSON,
few-shot videos with DensePose, instance maps)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'scripts'))


@pytest.mark.parametrize('name', ['spade', 'pix2pixHD', 'munit', 'funit', 'vid2vid_pose',
                                  'fs_vid2vid_pose'])
def test_train_from_lmdb(tmp_path, name):
    import build_lmdb
    import train
    from imaginaire_amd.utils.unit_test_data import lmdb_config, make_raw_dataset
    cfg = os.path.join(ROOT, 'configs', 'unit_test', name + '.yaml')
    raw, lmdb = str(tmp_path / 'raw'), str(tmp_path / 'lmdb')
    _, paired = make_raw_dataset(cfg, raw)
    lcfg = lmdb_config(cfg, lmdb, str(tmp_path / 'cfg.yaml'), max_iter=1)
    build_lmdb.main(['--config', lcfg, '--data_root', raw, '--output_root', lmdb] +
                    (['--paired'] if paired else []))
    assert os.path.exists(os.path.join(lmdb, 'all_filenames.json'))
    train.main(['--single_gpu', '--config', lcfg, '--logdir', str(tmp_path / 'logs')])
