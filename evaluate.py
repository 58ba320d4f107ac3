"""Evaluation entry point (reference evaluate.py:1-79): loads every ``*.pt``
checkpoint in ``--checkpoint_logdir`` in order and writes its metrics (FID)."""
import argparse
import glob
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from imaginaire_amd.config import Config  # noqa: E402
from imaginaire_amd.utils.cudnn import init_cudnn  # noqa: E402
from imaginaire_amd.utils.dataset import get_train_and_val_dataloader  # noqa: E402
from imaginaire_amd.utils.distributed import init_dist  # noqa: E402
from imaginaire_amd.utils.distributed import master_only_print as print  # noqa: E402
from imaginaire_amd.utils.gpu_affinity import set_affinity  # noqa: E402
from imaginaire_amd.utils.logging import init_logging, make_logging_dir  # noqa: E402
from imaginaire_amd.utils.trainer import (get_model_optimizer_and_scheduler, get_trainer,  # noqa
                                          set_random_seed)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description='Evaluation')
    p.add_argument('--config', required=True, help='Path to the training config file.')
    p.add_argument('--logdir', help='Dir for saving evaluation results.')
    p.add_argument('--checkpoint_logdir', required=True, help='Dir for loading models.')
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
    if not args.single_gpu and int(os.environ.get('WORLD_SIZE', '1')) > 1:
        cfg.local_rank = args.local_rank
        init_dist(cfg.local_rank)
    elif torch.cuda.is_available():
        torch.cuda.set_device(args.local_rank)
    if args.num_workers is not None:
        cfg.data.num_workers = args.num_workers
    cfg.date_uid, cfg.logdir = init_logging(args.config, args.logdir)
    make_logging_dir(cfg.logdir)
    init_cudnn(cfg.cudnn.deterministic, cfg.cudnn.benchmark)
    train_data_loader, val_data_loader = get_train_and_val_dataloader(cfg)
    net_G, net_D, opt_G, opt_D, sch_G, sch_D = get_model_optimizer_and_scheduler(cfg,
                                                                                seed=args.seed)
    trainer = get_trainer(cfg, net_G, net_D, opt_G, opt_D, sch_G, sch_D, train_data_loader,
                          val_data_loader)
    checkpoints = sorted(glob.glob('{}/*.pt'.format(args.checkpoint_logdir)))
    for checkpoint in checkpoints:
        current_epoch, current_iteration = trainer.load_checkpoint(cfg, checkpoint, resume=True)
        trainer.current_epoch = current_epoch
        trainer.current_iteration = current_iteration
        trainer.write_metrics()
    print('Done with evaluation!!!')


if __name__ == '__main__':
    main()
