"""Single-sample inference from files (portable version of the fork's
my_inference.py:1-129, which hard-codes Windows paths).

    python scripts/single_image_inference.py --config CFG --checkpoint CKPT \
        --label seg.tif --image img.npy --output out.png [--crop_w 512] [--repeat 2]

* ``--label``: 16-bit TIFF / PNG / .npy label map (uint16 scaled by 1/65535,
  uint8 by 1/255, HxWxC; channel order flipped to RGB for 3/4-channel images
  like the fork's OpenCV reader);
* ``--image``: optional .npy / image file used as the style image (kept in
  [0, 1], as the fork does);
* runs ``net_G.inference`` (EMA model when the config enables it) ``--repeat``
  times — the fork calls it twice so the frozen-eps style code is reused.
"""
import argparse
import os
import sys

import numpy as np
import torch
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imaginaire_amd.config import Config  # noqa: E402
from imaginaire_amd.utils.cudnn import init_cudnn  # noqa: E402
from imaginaire_amd.utils.misc import to_device  # noqa: E402
from imaginaire_amd.utils.trainer import (get_model_optimizer_and_scheduler, get_trainer,  # noqa
                                          set_random_seed)


def _read(path):
    if path.endswith('.npy'):
        return np.load(path, allow_pickle=False)
    img = np.array(Image.open(path))
    if img.ndim == 3 and img.shape[2] in (3, 4):
        pass  # PIL already returns RGB(A)
    return img


def _to_tensor(arr, crop_w=None):
    arr = np.asarray(arr)
    if arr.ndim == 2:
        arr = arr[:, :, None]
    if crop_w:
        arr = arr[:, :crop_w]
    if arr.dtype == np.uint16:
        arr = arr.astype(np.float32) / 65535.
    elif arr.dtype == np.uint8:
        arr = arr.astype(np.float32) / 255.
    return torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float32)).permute(2, 0, 1)[None]


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--config', required=True)
    p.add_argument('--checkpoint', required=True)
    p.add_argument('--label', required=True)
    p.add_argument('--image', default=None)
    p.add_argument('--output', required=True)
    p.add_argument('--crop_w', type=int, default=None)
    p.add_argument('--repeat', type=int, default=2)
    p.add_argument('--seed', type=int, default=0)
    args = p.parse_args(argv)
    set_random_seed(args.seed, by_rank=True)
    cfg = Config(args.config)
    if not hasattr(cfg, 'inference_args'):
        cfg.inference_args = None
    init_cudnn(cfg.cudnn.deterministic, cfg.cudnn.benchmark)
    nets = get_model_optimizer_and_scheduler(cfg, seed=args.seed)
    trainer = get_trainer(cfg, *nets, None, None)
    trainer.load_checkpoint(cfg, args.checkpoint)
    net_G = trainer.net_G.module.averaged_model if cfg.trainer.model_average \
        else trainer.net_G.module
    net_G.eval()
    data = {'label': _to_tensor(_read(args.label), args.crop_w), 'key': {'seg_maps': ['']}}
    if args.image:
        data['images'] = _to_tensor(_read(args.image), args.crop_w)
    device = next(net_G.parameters()).device
    data = to_device(data, device)
    kwargs = vars(cfg.inference_args) if cfg.inference_args is not None else {}
    with torch.no_grad():
        for _ in range(max(1, args.repeat)):
            output_images, _ = net_G.inference(data, **kwargs)
    image = ((output_images[0].float().clamp(-1, 1) + 1) * 0.5).cpu().numpy()
    image = np.transpose(image, (1, 2, 0)) * 255
    os.makedirs(os.path.dirname(os.path.abspath(args.output)), exist_ok=True)
    Image.fromarray(np.uint8(image[:, :, :3])).save(args.output)
    print('saved', args.output)


if __name__ == '__main__':
    main()
