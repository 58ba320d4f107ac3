"""Download + extract a public example dataset (reference scripts/download_dataset.py:1-49).

    python scripts/download_dataset.py --dataset afhq_dog2cat [--data_dir ./dataset]

Needs network access to Google Drive. Offline, use ``--synthetic CFG`` to write a raw
dataset of the same layout procedurally (scripts/make_unit_test_data.py).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _fetch import download_file_from_google_drive, safe_extract  # noqa: E402

DATASETS = {'afhq_dog2cat': '1XaiwS0eRctqm-JEDezOBy4TXriAQgc4_',
            'animal_faces': '1ftr1xWm0VakGlLUWi7-hdAt9W37luQOA'}


def main(argv=None):
    p = argparse.ArgumentParser(description='Download and process dataset')
    p.add_argument('--dataset', required=True, choices=sorted(DATASETS))
    p.add_argument('--data_dir', default='./dataset')
    p.add_argument('--synthetic', default=None, metavar='CFG',
                   help='offline: generate a synthetic raw dataset for CFG instead')
    args = p.parse_args(argv)
    folder = os.path.join(args.data_dir, args.dataset + '_raw')
    os.makedirs(args.data_dir, exist_ok=True)
    if args.synthetic:
        from imaginaire_amd.utils.unit_test_data import make_raw_dataset
        for split in ('train', 'test'):
            make_raw_dataset(args.synthetic, os.path.join(folder, split))
        print('synthetic raw dataset written to', folder)
        return
    archive = folder + '.tar.gz'
    if not os.path.exists(archive) and not os.path.exists(folder):
        print('Downloading the dataset {}.'.format(args.dataset))
        download_file_from_google_drive(DATASETS[args.dataset], archive)
    if not os.path.exists(folder):
        print('Extracting the dataset {}.'.format(args.dataset))
        safe_extract(archive, folder)


if __name__ == '__main__':
    main()
