"""FID evaluation throughput on a synthetic COCO-Stuff-shaped set (BASELINE.md "How the new
framework will be measured": SPADE 256x512 + FID on a synthetic set).

Runs the same path as ``SPADETrainer.write_metrics`` (reference trainers/spade.py:
_compute_fid; evaluation/fid.py:16-226): real-image Inception statistics, then generator
inference with a random style + Inception features for the fake statistics, then the Fréchet
distance (fp64 eigendecomposition on the GPU). Weights are random-init (no network for the
pretrained Inception / checkpoints), so the FID *value* only checks that the pipeline is
finite and deterministic; the number that matters is images/s through G + Inception.

    python scripts/bench_fid.py [--samples 512] [--batch 16] [--eager]

Prints one JSON line.
"""
import argparse
import functools
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


class _Loader(object):
    """Minimal data loader: a fixed number of synthetic device batches."""

    def __init__(self, src, n_batches):
        self.src, self.n_batches, self.batch_size = src, n_batches, src.batch_size
        self.dataset = range(n_batches * src.batch_size)

    def __len__(self):
        return self.n_batches

    def __iter__(self):
        for _ in range(self.n_batches):
            yield self.src.next()


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--config', default=os.path.join(HERE, 'configs', 'bench',
                                                    'spade_256x512_synthetic.yaml'))
    p.add_argument('--samples', type=int, default=512)
    p.add_argument('--batch', type=int, default=16)
    p.add_argument('--eager', action='store_true')
    args = p.parse_args()
    if args.eager:
        os.environ['IMAGINAIRE_AMD_EAGER'] = '1'
    import torch
    from imaginaire_amd.config import Config
    from imaginaire_amd.datasets.synthetic import DeviceBatchSource
    from imaginaire_amd.evaluation.fid import calculate_frechet_distance, get_inception_mean_cov
    from imaginaire_amd.utils.cudnn import init_cudnn
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer

    real_stdout, sys.stdout = sys.stdout, sys.stderr
    import threading

    def heartbeat(t0=time.time()):  # the eager path runs minutes without other output
        while True:
            time.sleep(20)
            print('[bench_fid] alive %.0f s' % (time.time() - t0), file=sys.__stderr__,
                  flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    torch.cuda.set_device(0)
    init_cudnn(False, True)
    device = torch.device('cuda', 0)
    cfg = Config(args.config)
    cfg.logdir = os.path.join('/tmp', 'imaginaire_amd_fid')
    net_G, net_D, opt_G, opt_D, sch_G, sch_D = get_model_optimizer_and_scheduler(cfg, seed=0)
    trainer = get_trainer(cfg, net_G, net_D, opt_G, opt_D, sch_G, sch_D,
                          train_data_loader=[], val_data_loader=None)
    n_batches = max(1, args.samples // args.batch)
    src = DeviceBatchSource(cfg, args.batch, device, pool=32, seed=123)
    preprocess = functools.partial(trainer._start_of_iteration, current_iteration=0)
    # A freshly initialised G is not evaluable: its spectral-norm u/v are random (sigma =
    # u^T W v can be ~0 -> inf weights) and its BatchNorm running stats are the defaults.
    # A few no-grad train-mode forwards (power iterations + running statistics) stand in for
    # training, as in the reference where FID is computed on a trained checkpoint.
    calib = 5
    with torch.no_grad(), trainer.autocast():
        net_G.train()
        for _ in range(calib):
            net_G(preprocess(src.next()), random_style=True)
    net_G.eval()
    gen = functools.partial(net_G, random_style=True)

    def stats(generator, n):
        src.step = 0
        loader = _Loader(src, n)
        with torch.no_grad(), trainer.autocast():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mean, cov = get_inception_mean_cov(loader, 'images', 'fake_images', generator,
                                               None, preprocess)
            torch.cuda.synchronize()
        return mean, cov, time.perf_counter() - t0

    stats(gen, 1)  # warm-up: kernels, Inception build, MIOpen/k11 tuning
    real_mean, real_cov, t_real = stats(None, n_batches)
    fake_mean, fake_cov, t_fake = stats(gen, n_batches)
    t0 = time.perf_counter()
    fid = calculate_frechet_distance(real_mean, real_cov, fake_mean, fake_cov)
    t_fd = time.perf_counter() - t0
    # determinism: the same statistics again give the same distance
    fid2 = calculate_frechet_distance(real_mean, real_cov, fake_mean, fake_cov)
    n = n_batches * args.batch
    sys.stdout = real_stdout
    print(json.dumps({
        'metric': 'FID evaluation throughput (SPADE 256x512 G inference + Inception-v3 pool3)',
        'value': round(n / t_fake, 2), 'unit': 'images/s', 'n_gpus': 1, 'samples': n,
        'batch': args.batch, 'real_stats_img_s': round(n / t_real, 2),
        'frechet_distance_s': round(t_fd, 3), 'fid_random_init': round(float(fid), 4),
        'fid_repeat_equal': bool(float(fid) == float(fid2)), 'g_calibration_steps': calib,
        'dtype': 'bf16', 'data': 'synthetic COCO-Stuff-shaped, random-init G and Inception',
        'kernels': 'eager-reference' if args.eager else 'hip'}), flush=True)


if __name__ == '__main__':
    main()
