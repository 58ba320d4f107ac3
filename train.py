"""Training entry point (reference train.py:1-93).

    python train.py --config configs/bench/spade_256x512_synthetic.yaml [--logdir D]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py --config ...

One process per GPU; RCCL (``nccl``) process group on GPU, gloo on CPU hosts.
"""
import argparse
import faulthandler
import os
import sys

import torch

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from imaginaire_amd.config import Config  # noqa: E402
from imaginaire_amd.utils.cudnn import init_cudnn  # noqa: E402
from imaginaire_amd.utils.dataset import get_train_and_val_dataloader  # noqa: E402
from imaginaire_amd.utils.distributed import init_dist, get_world_size  # noqa: E402
from imaginaire_amd.utils.distributed import master_only_print as print  # noqa: E402
from imaginaire_amd.utils.health import FaultInjector, StragglerMonitor, Watchdog  # noqa: E402
from imaginaire_amd.utils.logging import init_logging, make_logging_dir  # noqa: E402
from imaginaire_amd.utils.trainer import (get_model_optimizer_and_scheduler, get_trainer,  # noqa
                                          set_random_seed)


def parse_args(argv=None):
    parser = argparse.ArgumentParser(description='Training')
    parser.add_argument('--config', required=True, help='Path to the training config file.')
    parser.add_argument('--logdir', help='Dir for saving logs and models.')
    parser.add_argument('--checkpoint', default='', help='Checkpoint path.')
    parser.add_argument('--seed', type=int, default=2, help='Random seed.')
    parser.add_argument('--local_rank', '--local-rank', type=int,
                        default=int(os.environ.get('LOCAL_RANK', 0)))
    parser.add_argument('--single_gpu', action='store_true')
    parser.add_argument('--num_workers', type=int)
    parser.add_argument('--backend', default=None, help='nccl (RCCL) / gloo; default auto')
    parser.add_argument('--no_graph', '--no-graph', action='store_true',
                        help='run every iteration eagerly (no hipGraph replay)')
    parser.add_argument('--watchdog_timeout', '--watchdog-timeout', type=float,
                        default=float(os.environ.get('IMAGINAIRE_AMD_WATCHDOG_S', 900)),
                        help='seconds without a finished iteration before the rank dumps its '
                             'stacks to <logdir>/hang_rank<R>.txt and exits (0: off)')
    parser.add_argument('--watchdog_grace', '--watchdog-grace', type=float, default=None,
                        help='bound for start-up, checkpoint / FID phases and the first '
                             'iterations of an epoch (default 10x --watchdog-timeout)')
    return parser.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    set_random_seed(args.seed, by_rank=True)
    cfg = Config(args.config)
    if not args.single_gpu and int(os.environ.get('WORLD_SIZE', '1')) > 1:
        cfg.local_rank = args.local_rank
        init_dist(cfg.local_rank, backend=args.backend)
    elif torch.cuda.is_available():
        torch.cuda.set_device(args.local_rank)
    if args.num_workers is not None:
        cfg.data.num_workers = args.num_workers
    cfg.date_uid, cfg.logdir = init_logging(args.config, args.logdir)
    make_logging_dir(cfg.logdir)
    init_cudnn(cfg.cudnn.deterministic, cfg.cudnn.benchmark)
    train_data_loader, val_data_loader = get_train_and_val_dataloader(cfg, seed=args.seed)
    net_G, net_D, opt_G, opt_D, sch_G, sch_D = get_model_optimizer_and_scheduler(cfg,
                                                                                seed=args.seed)
    trainer = get_trainer(cfg, net_G, net_D, opt_G, opt_D, sch_G, sch_D, train_data_loader,
                          val_data_loader)
    current_epoch, current_iteration = trainer.load_checkpoint(cfg, args.checkpoint)
    # the D -> G iteration; replayed from a hipGraph after a few eager iterations when the
    # trainer supports it (single process, see imaginaire_amd/utils/cuda_graph.py)
    from imaginaire_amd.utils.cuda_graph import make_trainer_step
    train_step, _ = make_trainer_step(trainer, enabled=not args.no_graph)
    # failure detection (imaginaire_amd/utils/health.py): per-rank hang watchdog, optional
    # fault injection, straggler report at logging boundaries
    faults = FaultInjector()
    stragglers = StragglerMonitor()
    start_iteration = current_iteration
    with Watchdog(args.watchdog_timeout, cfg.logdir,
                  first_timeout=args.watchdog_grace) as watchdog:
        watchdog.beat(current_iteration, 'start')
        for epoch in range(current_epoch, cfg.max_epoch):
            print('Epoch {} ...'.format(epoch))
            if hasattr(train_data_loader.sampler, 'set_epoch'):
                train_data_loader.sampler.set_epoch(current_epoch)
            # epoch start-up (loader workers, temporal-curriculum / local-enhancer switches,
            # first use of new shapes) runs until the epoch's first iteration ends under the
            # long grace bound
            watchdog.beat(current_iteration, 'start of epoch %d' % epoch, grace=True)
            trainer.start_of_epoch(current_epoch)
            for it, data in enumerate(train_data_loader):
                data = trainer.start_of_iteration(data, current_iteration)
                if faults:
                    data = faults.apply(current_iteration, data)
                train_step(data)
                current_iteration += 1
                # snapshot save + FID (write_metrics) may run here: long bound
                watchdog.beat(current_iteration, 'end_of_iteration', grace=True)
                trainer.end_of_iteration(data, current_epoch, current_iteration)
                # the first iteration of an epoch and the hipGraph warm-up / capture
                # iterations of the run keep the long bound as well
                watchdog.beat(current_iteration, grace=(it == 0 or
                                                        current_iteration < start_iteration + 5))
                stragglers.tick()
                if get_world_size() > 1 and current_iteration % cfg.logging_iter == 0:
                    stragglers.report()
                if current_iteration >= cfg.max_iter:
                    print('Done with training!!!')
                    return
            current_epoch += 1
            with watchdog.grace(current_iteration, 'end_of_epoch'):
                trainer.end_of_epoch(data, current_epoch, current_iteration)
    print('Done with training!!!')


if __name__ == "__main__":
    main()
