"""IO helpers (reference utils/io.py:14-122).

There is no network on MI355X training boxes here, so ``get_checkpoint`` only
resolves locally cached files (``$TORCH_HOME/checkpoints``) and fails with a
clear message otherwise; everything else matches the reference.
"""
import os

import torch.distributed as dist

from imaginaire_amd.utils.distributed import is_master


def save_pilimage_in_jpeg(fullname, output_img):
    dirname = os.path.dirname(fullname)
    if dirname:
        os.makedirs(dirname, exist_ok=True)
    output_img.save(fullname, 'JPEG', quality=99)


def save_intermediate_training_results(visualization_images, logdir, current_epoch,
                                       current_iteration):
    from imaginaire_amd.utils.visualization.common import save_image_grid
    visualization_images = (visualization_images + 1) / 2
    output_filename = os.path.join(logdir, 'images', 'epoch_{:05}iteration{:09}.jpg'.format(
        current_epoch, current_iteration))
    save_image_grid(visualization_images, output_filename, nrow=1)


def get_confirm_token(response):
    """Google-Drive large-file confirmation token from the response cookies (io.py:62-75)."""
    for key, value in response.cookies.items():
        if key.startswith('download_warning'):
            return value
    return None


def save_response_content(response, destination, chunk_size=32768):
    """Stream a ``requests`` response body to ``destination`` (io.py:78-90)."""
    with open(destination, 'wb') as f:
        for chunk in response.iter_content(chunk_size):
            if chunk:
                f.write(chunk)


def download_file_from_google_drive(file_id, destination):
    try:
        import requests
    except ImportError:
        raise RuntimeError('requests is not available to download {}'.format(file_id))
    url = "https://docs.google.com/uc?export=download"
    session = requests.Session()
    response = session.get(url, params={'id': file_id}, stream=True)
    token = get_confirm_token(response)
    if token:
        response = session.get(url, params={'id': file_id, 'confirm': token}, stream=True)
    save_response_content(response, destination)


def get_checkpoint(checkpoint_path, url='', allow_download=False):
    if 'TORCH_HOME' not in os.environ:
        os.environ['TORCH_HOME'] = os.getcwd()
    save_dir = os.path.join(os.environ['TORCH_HOME'], 'checkpoints')
    os.makedirs(save_dir, exist_ok=True)
    full_checkpoint_path = os.path.join(save_dir, checkpoint_path)
    if not os.path.exists(full_checkpoint_path):
        if not allow_download:
            raise FileNotFoundError(
                'checkpoint {} not found locally and downloads are disabled'.format(
                    full_checkpoint_path))
        os.makedirs(os.path.dirname(full_checkpoint_path), exist_ok=True)
        if is_master():
            download_file_from_google_drive(url, full_checkpoint_path)
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
    return full_checkpoint_path
