"""Download per-model inference test data (reference scripts/download_test_data.py:1-53).

    python scripts/download_test_data.py --model_name spade

Writes ``projects/<model>/test_data``. Needs network access; offline, pass
``--synthetic CFG`` to generate test inputs of the config's layout instead.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _fetch import download_file_from_google_drive, safe_extract  # noqa: E402

URLS = {
    'pix2pixhd': '1Xg9m184zkuG8H0LHdBtSzt2VbMi3SWwR',
    'spade': '1ESm-gHWu_aMHnKF42qkGc8qf1SBECsgf',
    'funit': '1a-EE_6RsYPUoKxEl5oXrpRmKYUltqaD-',
    'coco_funit': '1JYVYB0Q1VStDLOb0SBJbN1vkaf6KrGDh',
    'unit': '17BbwnCG7qF7FI-t9VkORv2XCKqlrY1CO',
    'munit': '1VPgHGuQfmm1N1Vh56wr34wtAwaXzjXtH',
    'vid2vid': '1SHvGPMq-55GDUQ0Ac2Ng0eyG5xCPeKhc',
    'fs_vid2vid': '1fTj0HHjzcitgsSeG5O_aWMF8yvCQUQkN',
    'wc_vid2vid_cityscapes': '1KKzrTHfbpBY9xtLqK8e3QvX8psSdrFcD',
    'wc_vid2vid_mannequin': '1mafZf9KJrwUGGI1kBTvwgehHSqP5iaA0',
}


def main(argv=None):
    p = argparse.ArgumentParser(description='Download test data.')
    p.add_argument('--model_name', required=True, choices=sorted(URLS))
    p.add_argument('--synthetic', default=None, metavar='CFG')
    args = p.parse_args(argv)
    test_data_dir = os.path.join('projects', args.model_name, 'test_data')
    if os.path.exists(test_data_dir):
        print('Test data exists at', test_data_dir)
        return
    if args.synthetic:
        from imaginaire_amd.utils.unit_test_data import make_raw_dataset
        make_raw_dataset(args.synthetic, test_data_dir)
        print('synthetic test data written to', test_data_dir)
        return
    os.makedirs(test_data_dir, exist_ok=True)
    archive = test_data_dir + '.tar.gz'
    if not os.path.exists(archive):
        print('Downloading test data to', archive)
        download_file_from_google_drive(URLS[args.model_name], archive)
    print('Extracting test data to', test_data_dir)
    safe_extract(archive, test_data_dir)


if __name__ == '__main__':
    main()
