"""Inference entry point (reference inference.py:1-91).

    python inference.py --config CFG --checkpoint CKPT --output_dir OUT [--single_gpu]

Runs ``trainer.test`` on ``cfg.test_data`` and writes the generated images.
There is no network access: ``--checkpoint`` must point at a local file
(``cfg.pretrained_weight`` downloads are only attempted when
``IMAGINAIRE_AMD_ALLOW_DOWNLOAD=1``).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from imaginaire_amd.config import Config  # noqa: E402
from imaginaire_amd.utils.cudnn import init_cudnn  # noqa: E402
from imaginaire_amd.utils.dataset import get_test_dataloader  # noqa: E402
from imaginaire_amd.utils.distributed import init_dist  # noqa: E402
from imaginaire_amd.utils.gpu_affinity import set_affinity  # noqa: E402
from imaginaire_amd.utils.io import get_checkpoint  # noqa: E402
from imaginaire_amd.utils.logging import init_logging  # noqa: E402
from imaginaire_amd.utils.trainer import (get_model_optimizer_and_scheduler, get_trainer,  # noqa
                                          set_random_seed)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description='Inference')
    p.add_argument('--config', required=True, help='Path to the training config file.')
    p.add_argument('--checkpoint', default='', help='Checkpoint path.')
    p.add_argument('--output_dir', required=True, help='Location to save the image outputs')
    p.add_argument('--logdir', help='Dir for saving logs and models.')
    p.add_argument('--seed', type=int, default=0, help='Random seed.')
    p.add_argument('--local_rank', '--local-rank', type=int,
                   default=int(os.environ.get('LOCAL_RANK', 0)))
    p.add_argument('--single_gpu', action='store_true')
    p.add_argument('--num_workers', type=int)
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    set_affinity(args.local_rank)
    set_random_seed(args.seed, by_rank=True)
    cfg = Config(args.config)
    if not hasattr(cfg, 'inference_args'):
        cfg.inference_args = None
    if not args.single_gpu and int(os.environ.get('WORLD_SIZE', '1')) > 1:
        cfg.local_rank = args.local_rank
        init_dist(cfg.local_rank)
    elif torch.cuda.is_available():
        torch.cuda.set_device(args.local_rank)
    if args.num_workers is not None:
        cfg.data.num_workers = args.num_workers
    cfg.date_uid, cfg.logdir = init_logging(args.config, args.logdir)
    init_cudnn(cfg.cudnn.deterministic, cfg.cudnn.benchmark)
    test_data_loader = get_test_dataloader(cfg)
    net_G, net_D, opt_G, opt_D, sch_G, sch_D = get_model_optimizer_and_scheduler(cfg,
                                                                                seed=args.seed)
    trainer = get_trainer(cfg, net_G, net_D, opt_G, opt_D, sch_G, sch_D, None, test_data_loader)
    if args.checkpoint == '':
        url = getattr(cfg, 'pretrained_weight', '')
        if not url:
            raise ValueError('no --checkpoint given and cfg.pretrained_weight is empty')
        args.checkpoint = get_checkpoint(args.config.replace('.yaml', '.pt'), url)
    trainer.load_checkpoint(cfg, args.checkpoint)
    trainer.current_epoch = -1
    trainer.current_iteration = -1
    os.makedirs(args.output_dir, exist_ok=True)
    trainer.test(test_data_loader, args.output_dir, cfg.inference_args)


if __name__ == '__main__':
    main()
