"""Write a synthetic raw folder dataset for a config (reference scripts/download_test_data.py
and the ``dataset/unit_test/raw`` fixtures used by scripts/test_training.sh).

    python scripts/make_unit_test_data.py --config CFG --output_root dataset/unit_test/raw/X \
        [--lmdb_root dataset/unit_test/lmdb/X --lmdb_config out.yaml]

Prints ``paired=<0|1>`` (the ``--paired`` flag build_lmdb.py needs). With
``--lmdb_root``/``--lmdb_config`` it also writes a copy of CFG whose splits read
that LMDB (synthetic dataset types replaced by the real dataset classes).
"""
import argparse
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imaginaire_amd.utils.unit_test_data import lmdb_config, make_raw_dataset  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--config', required=True)
    p.add_argument('--output_root', required=True)
    p.add_argument('--num_sequences', type=int, default=2)
    p.add_argument('--frames', type=int, default=None)
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--size', type=str, default=None, help='H,W of the raw images')
    p.add_argument('--lmdb_root', default=None)
    p.add_argument('--lmdb_config', default=None)
    p.add_argument('--max_iter', type=int, default=None)
    args = p.parse_args(argv)
    if os.path.exists(args.output_root):
        shutil.rmtree(args.output_root)
    size = tuple(int(x) for x in args.size.split(',')) if args.size else None
    _, paired = make_raw_dataset(args.config, args.output_root, args.num_sequences,
                                 args.frames, args.seed, size)
    if args.lmdb_config:
        lmdb_config(args.config, args.lmdb_root, args.lmdb_config, args.max_iter)
    print('paired=%d' % int(paired))
    return paired


if __name__ == '__main__':
    main()
