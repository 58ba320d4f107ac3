"""Folder -> LMDB dataset conversion (reference scripts/build_lmdb.py:1-125).

    python scripts/build_lmdb.py --config CFG --data_root DIR --output_root OUT [--paired]

Writes ``<OUT>/<data_type>/data.mdb`` (native writer, csrc/lmdb_io.cpp),
``<OUT>/all_filenames.json`` and ``<OUT>/metadata.json``.
"""
import argparse
import copy
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imaginaire_amd.config import Config  # noqa: E402
from imaginaire_amd.utils.lmdb import (build_lmdb, check_and_add, construct_file_path,  # noqa
                                       create_metadata)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description='Folder -> LMDB conversion')
    p.add_argument('--data_root', type=str, required=True, help='Input data location.')
    p.add_argument('--config', type=str, required=True, help='Config with label info.')
    p.add_argument('--output_root', type=str, required=True, help='Output LMDB location')
    p.add_argument('--input_list', type=str, default='', help='list of images to use.')
    p.add_argument('--metadata_factor', type=float, default=0.75,
                   help='kept for CLI compatibility (the writer sizes files exactly)')
    p.add_argument('--overwrite', default=False, action='store_true')
    p.add_argument('--paired', default=False, action='store_true')
    p.add_argument('--large', default=False, action='store_true')
    p.add_argument('--remove_missing', default=False, action='store_true')
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    cfg = Config(args.config)
    if os.path.exists(args.output_root):
        if not args.overwrite:
            print('Output root LMDB already exists. Use --overwrite. Exiting...')
            return
        print('Deleting existing output LMDB.')
        shutil.rmtree(args.output_root)
    all_filenames, extensions = create_metadata(data_root=args.data_root, cfg=cfg,
                                                paired=args.paired, input_list=args.input_list)
    os.makedirs(args.output_root)
    for data_type in cfg.data.data_types:
        filepaths, keys = [], []
        filenames = all_filenames if args.paired else all_filenames[data_type]
        for sequence in filenames:
            for filename in copy.deepcopy(filenames[sequence]):
                fp = construct_file_path(args.data_root, data_type, sequence, filename,
                                         extensions[data_type])
                size = check_and_add(fp, '%s/%s' % (sequence, filename), filepaths, keys,
                                     remove_missing=args.remove_missing)
                if size == -1 and args.paired and args.remove_missing:
                    print('Removing %s from list' % filename)
                    filenames[sequence].remove(filename)
        if args.paired and args.remove_missing:
            for sequence in copy.deepcopy(all_filenames):
                if not all_filenames[sequence]:
                    all_filenames.pop(sequence)
        build_lmdb(filepaths, keys, os.path.join(args.output_root, data_type), None, args.large)
    with open(os.path.join(args.output_root, 'all_filenames.json'), 'w') as f:
        json.dump(all_filenames, f, indent=4)
    with open(os.path.join(args.output_root, 'metadata.json'), 'w') as f:
        json.dump(extensions, f, indent=4)


if __name__ == '__main__':
    main()
