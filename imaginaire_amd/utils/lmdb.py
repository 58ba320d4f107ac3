"""Folder <-> LMDB dataset utilities (reference utils/lmdb.py:14-215).

LMDB files are written by the framework's native writer
(``imaginaire_amd._C.lmdb_write``, csrc/lmdb_io.cpp) — one environment
directory per data type with ``data.mdb`` holding ``"<sequence>/<filename>"``
→ raw file bytes, exactly the reference layout.
"""
import glob
import os

from imaginaire_amd.utils import path
from imaginaire_amd.utils.distributed import master_only_print as print


def construct_file_path(root, data_type, sequence, filename, ext):
    return '%s/%s/%s/%s.%s' % (root, data_type, sequence, filename, ext)


def check_and_add(filepath, key, filepaths, keys, remove_missing=False):
    if not os.path.exists(filepath):
        print(filepath + ' does not exist.')
        if remove_missing:
            return -1
        raise FileNotFoundError(filepath + ' does not exist.')
    filepaths.append(filepath)
    keys.append(key)
    return os.path.getsize(filepath)


def write_entry(txn, key, filepath):
    """Put the raw bytes of ``filepath`` under ``key`` into a transaction-like object with a
    ``put(bytes, bytes)`` method (reference utils/lmdb.py:43-53)."""
    with open(filepath, 'rb') as f:
        data = f.read()
    txn.put(key.encode('ascii'), data)


def build_lmdb(filepaths, keys, output_filepath, map_size=None, large=False, page_size=4096):
    """Write one LMDB environment from (file, key) pairs. ``map_size`` / ``large``
    are accepted for interface parity; the native writer sizes the file exactly."""
    from imaginaire_amd.ops import _ext
    print('Writing LMDB to:', output_filepath)
    items = []
    for filepath, key in zip(filepaths, keys):
        with open(filepath, 'rb') as f:
            items.append((key.encode('ascii'), f.read()))
    _ext.ext().lmdb_write(output_filepath, items, page_size)


def get_all_filenames_from_list(list_name):
    with open(list_name, 'rt') as f:
        lines = [line.strip() for line in f.readlines()]
    all_filenames = dict()
    for line in lines:
        if '/' in line:
            folder_name = os.path.join(*line.split('/')[0:-1])
            image_name = line.split('/')[-1].replace('.jpg', '')
        else:
            folder_name, image_name = '.', line.replace('.jpg', '')
        all_filenames.setdefault(folder_name, []).append(image_name)
    return all_filenames


def get_lmdb_data_types(cfg):
    data_types, extensions = [], []
    for data_type in cfg.data.input_types:
        name = list(data_type.keys())
        assert len(name) == 1
        name = name[0]
        info = data_type[name]
        if getattr(info, 'computed_on_the_fly', False):
            continue
        data_types.append(name)
        extensions.append(info['ext'] if 'ext' in info else None)
    cfg.data.data_types = data_types
    cfg.data.extensions = extensions
    return cfg


def _list_sequence(data_root, data_type, sequence, ext):
    files = sorted(glob.glob('%s/%s/%s/*.%s' % (data_root, data_type, sequence, ext)))
    return [os.path.splitext(os.path.basename(f))[0] for f in files]


def create_metadata(data_root=None, cfg=None, paired=None, input_list=''):
    """File lists (+ extension map) of a folder dataset root."""
    cfg = get_lmdb_data_types(cfg)
    available = path.get_immediate_subdirectories(data_root)
    required = cfg.data.data_types
    missing = set(required) - set(available)
    assert not missing, '%s missing' % missing
    extensions = dict(zip(required, cfg.data.extensions))
    print('Data file extensions:', extensions)
    if paired:
        if input_list != '':
            all_filenames = get_all_filenames_from_list(input_list)
        else:
            if 'data_keypoint' in required:
                search_dir = 'data_keypoint'
            elif 'data_segmaps' in required:
                search_dir = 'data_segmaps'
            else:
                search_dir = required[0]
            print('Searching in dir: %s' % search_dir)
            sequences = path.get_recursive_subdirectories(os.path.join(data_root, search_dir),
                                                          extensions[search_dir])
            print('Found %d sequences' % len(sequences))
            all_filenames = {s: _list_sequence(data_root, search_dir, s, extensions[search_dir])
                             for s in sequences}
            print('Found %d files' % sum(len(v) for v in all_filenames.values()))
    else:
        all_filenames = {}
        for data_type in required:
            sequences = path.get_recursive_subdirectories(os.path.join(data_root, data_type),
                                                          extensions[data_type])
            all_filenames[data_type] = {
                s: _list_sequence(data_root, data_type, s, extensions[data_type])
                for s in sequences}
            print('Data type: %s, Found %d sequences, Found %d files' % (
                data_type, len(sequences),
                sum(len(v) for v in all_filenames[data_type].values())))
    return all_filenames, extensions
