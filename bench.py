"""Flagship benchmark: SPADE/GauGAN training throughput, 256x512, bf16.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Metric (BASELINE.json): whole-node images/s for SPADE 256x512 — one "step" is
one full training iteration of the reference SPADE trainer: D update (G
forward under no_grad, D forward on real+fake, hinge loss, backward, Adam)
followed by G update (G forward with style encoder, D forward, GAN + feature
matching + VGG-19 perceptual + KL, backward through D and G, Adam) and the EMA
update of the averaged generator. COCO-Stuff-shaped synthetic data
(183 classes + don't-care + edge), random-init weights, batch 4 per GPU
(the reference recipe), weak scaling. rank 0 prints ONE JSON line.
"""
import argparse
import contextlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

# Reference throughput: the model zoo trained SPADE COCO-Stuff 256x256 on a
# DGX-1 (8x V100) in 2-3 weeks => 26-39 img/s/node; pixel-scaled to 256x512
# => 13-20 img/s per 8-GPU node. We compare against the upper
# end (20 img/s), the conservative choice.
BASELINE_IMG_S = 20.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1,
                   help='number of ranks (one per GPU). Without a launcher (no WORLD_SIZE) '
                        'bench.py starts them itself through torch.distributed.run')
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=6)
    p.add_argument('--config', default=os.path.join(HERE, 'configs', 'bench',
                                                     'spade_256x512_synthetic.yaml'))
    p.add_argument('--batch', type=int, default=None, help='per-GPU batch (default: config)')
    p.add_argument('--eager', action='store_true',
                   help='self-baseline: PyTorch reference ops instead of the HIP kernels '
                        '(implies --no-graph)')
    p.add_argument('--no-graph', action='store_true',
                   help='issue every kernel from Python each step instead of replaying the '
                        'hipGraph-captured step (A/B)')
    p.add_argument('--profile-phases', action='store_true')
    p.add_argument('--verbose', action='store_true')
    p.add_argument('--backend', default='nccl',
                   help='process-group backend for N>1 (nccl = RCCL over xGMI; gloo for '
                        'single-GPU multi-rank rehearsals with --share-gpu)')
    p.add_argument('--device', default='cuda', choices=('cuda', 'cpu'),
                   help='cpu: plumbing rehearsal of the launcher / DDP path (gloo), no GPU')
    p.add_argument('--force-dist', action='store_true',
                   help='measurement only: run the distributed wrappers (bucketed DDP over a '
                        'native RCCL communicator, sync-BN exchanges) on a ONE-rank process '
                        'group, to price their overhead against the plain world-1 step')
    p.add_argument('--share-gpu', action='store_true',
                   help='testing only: every rank uses cuda:0 (rehearse the DDP path on one GPU)')
    p.add_argument('--torch-profile', action='store_true',
                   help='after warm-up, profile one step on the host (torch.profiler, CPU '
                        'activities) and print the top operators to stderr')
    p.add_argument('--conv-profile', action='store_true',
                   help='after warm-up, profile one step with device activity and shapes and '
                        'print GPU time per (op, input shapes) to stderr')
    p.add_argument('--op-profile', action='store_true',
                   help='like --conv-profile but for every aten op (self device time)')
    p.add_argument('--conv-log', action='store_true',
                   help='after warm-up, time every conv kernel call of one eager step (device '
                        'events) and print time / TF/s per (kind, shape, kernel) to stderr')
    p.add_argument('--op-stack', action='store_true',
                   help='with --op-profile: group the small elementwise ops by Python call site')
    return p.parse_args()


def _heartbeat(period=20.0):
    """Print a line to stderr every ``period`` s: the first warm-up step on a fresh
    box spends minutes inside MIOpen kernel compilation and prints nothing else."""
    import threading

    t0 = time.time()

    def run():
        while True:
            time.sleep(period)
            print('[bench] alive %.0f s' % (time.time() - t0), file=sys.__stderr__, flush=True)

    threading.Thread(target=run, daemon=True).start()


def _free_port():
    import socket
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """``--gpus N`` without a launcher: start N ranks (one process per GPU) as a CHILD
    ``torch.distributed.run`` and exit with its status. Runs before anything touches the
    GPU (no exec from a process holding a HIP context). Reference launch form:
    ``python -m torch.distributed.launch --nproc_per_node=N train.py`` (projects/*/README.md)."""
    import subprocess
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node=%d' % args.gpus, '--master-addr=127.0.0.1',
           '--master-port=%d' % _free_port(), os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    env.setdefault('OMP_NUM_THREADS', '4')
    print('[bench] launching %d ranks: %s' % (args.gpus, ' '.join(cmd)), file=sys.stderr,
          flush=True)
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    world_env = os.environ.get('WORLD_SIZE')
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    if world_env is not None and int(world_env) != args.gpus:
        sys.exit('bench.py: --gpus %d but WORLD_SIZE=%s: refusing to report a %s-rank number '
                 'as %d GPUs' % (args.gpus, world_env, world_env, args.gpus))
    if args.share_gpu and args.gpus > 1 and args.backend == 'nccl':
        sys.exit('bench.py: --share-gpu needs --backend gloo (RCCL cannot place two ranks '
                 'on one GPU)')
    _heartbeat()
    if args.eager:
        os.environ['IMAGINAIRE_AMD_EAGER'] = '1'
    import torch
    import torch.distributed as dist

    real_stdout = sys.stdout
    sys.stdout = sys.stderr  # keep stdout for the single JSON line
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if args.share_gpu:
        local_rank = 0
    from imaginaire_amd.config import Config
    from imaginaire_amd.utils.distributed import init_dist
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer
    from imaginaire_amd.datasets.synthetic import DeviceBatchSource

    on_gpu = args.device == 'cuda'
    if on_gpu:
        # set the device before the process group so RCCL binds rank r to GPU r
        torch.cuda.set_device(local_rank)
    if args.force_dist and world == 1:
        os.environ.setdefault('RANK', '0')
        os.environ.setdefault('WORLD_SIZE', '1')
        os.environ.setdefault('MASTER_PORT', str(29500 + os.getpid() % 1000))
        os.environ['IMAGINAIRE_AMD_FORCE_DIST'] = '1'
    if world > 1 or args.force_dist:
        init_dist(local_rank, backend=args.backend if on_gpu else 'gloo')
    from imaginaire_amd.utils.cudnn import init_cudnn
    init_cudnn(False, True)
    device = torch.device('cuda', local_rank) if on_gpu else torch.device('cpu')
    cfg = Config(args.config)
    cfg.logdir = os.path.join('/tmp', 'imaginaire_amd_bench')
    if args.batch:
        cfg.data.train.batch_size = args.batch
    if args.profile_phases:
        cfg.speed_benchmark = True  # synchronised per-phase timers in the trainer
    bs = cfg.data.train.batch_size
    net_G, net_D, opt_G, opt_D, sch_G, sch_D = get_model_optimizer_and_scheduler(cfg, seed=0)
    trainer = get_trainer(cfg, net_G, net_D, opt_G, opt_D, sch_G, sch_D,
                          train_data_loader=[], val_data_loader=None)
    src = DeviceBatchSource(cfg, bs, device, pool=8, seed=rank)
    # steady-state iteration: hipGraph-captured (world size 1) after max(1, W-2) eager
    # warm-up steps, so with W >= 2 the timed steps are all replays
    from imaginaire_amd.utils.cuda_graph import make_trainer_step
    use_graph = on_gpu and not (args.no_graph or args.eager or args.profile_phases or
                                args.conv_log) and args.warmup >= 2
    run_step, graphed = make_trainer_step(trainer, warmup=min(3, max(1, args.warmup - 2)),
                                          enabled=use_graph)

    def step(it):
        data = src.next()
        data = trainer.start_of_iteration(data, it)
        run_step(data)

    for it in range(args.warmup):
        step(it)
        if rank == 0:
            print('[bench] warmup {} done'.format(it), flush=True)

    if args.torch_profile and rank == 0:
        from torch.profiler import ProfilerActivity, profile
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU], with_stack=False) as prof:
            step(args.warmup)
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by='self_cpu_time_total', row_limit=45),
              flush=True)

    if args.conv_log and rank == 0:
        from imaginaire_amd.ops import conv as conv_ops
        torch.cuda.synchronize()
        conv_ops.enable_conv_log(True)
        t0 = time.perf_counter()
        step(args.warmup)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        rows = conv_ops.conv_log_summary()
        conv_ops.enable_conv_log(False)
        tot = sum(r[4] for r in rows)
        fl = sum(r[5] * r[4] * 1e9 for r in rows)
        print('conv kernels in one eager step: %.2f ms of %.1f ms wall, %.1f TFLOP, %.0f TF/s' % (
            tot, wall, fl / 1e12, fl / max(tot, 1e-9) / 1e9))
        by_kind = {}
        for r in rows:
            k = by_kind.setdefault((r[0], r[1]), [0, 0.0, 0.0])
            k[0] += r[3]
            k[1] += r[4]
            k[2] += r[5] * r[4] * 1e9
        for (kind, path), (n, ms, f) in sorted(by_kind.items(), key=lambda kv: -kv[1][1]):
            print('  %-6s %-7s %4d calls %8.2f ms %6.0f TF/s' % (kind, path, n, ms,
                                                              f / max(ms, 1e-9) / 1e9))
        for kind, path, desc, n, ms, tfs in rows:
            print('%8.3f ms %3d  %-6s %-7s %5.0f TF/s  %s' % (ms, n, kind, path, tfs, desc))
        sys.stdout.flush()

    if (args.conv_profile or args.op_profile) and rank == 0:
        from torch.profiler import ProfilerActivity, profile
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                     record_shapes=True, with_stack=args.op_stack) as prof:
            step(args.warmup)
            torch.cuda.synchronize()
        if args.op_profile and args.op_stack:
            rows = [e for e in prof.key_averages(group_by_stack_n=4)
                    if e.self_device_time_total > 0 and e.key.startswith('aten::') and
                    e.key not in ('aten::convolution_backward', 'aten::miopen_convolution')]
            rows.sort(key=lambda e: -e.self_device_time_total)
            print('op self GPU time by call site (aten ops only): %.2f ms' % (
                sum(e.self_device_time_total for e in rows) / 1e3))
            for e in rows[:60]:
                print('%9.3f ms %5d  %-24s %s' % (e.self_device_time_total / 1e3, e.count,
                                                  e.key[:24], ' <- '.join(e.stack[:4])[:220]))
        elif args.op_profile:
            rows = [e for e in prof.key_averages(group_by_input_shape=True)
                    if e.self_device_time_total > 0 and e.input_shapes is not None and
                    not e.key.startswith(('void', 'igemm', 'iamd', '__amd', 'Sub'))]
            rows.sort(key=lambda e: -e.self_device_time_total)
            tot = sum(e.self_device_time_total for e in rows)
            print('op self GPU time in one step: %.2f ms' % (tot / 1e3))
            for e in rows[:250]:
                print('%9.3f ms %4d  %-34s %s' % (e.self_device_time_total / 1e3, e.count,
                                                  e.key[:34], str(e.input_shapes)[:140]))
        else:
            rows = [e for e in prof.key_averages(group_by_input_shape=True)
                    if e.key in ('aten::convolution', 'aten::convolution_backward')]
            rows.sort(key=lambda e: -e.device_time_total)
            tot = sum(e.device_time_total for e in rows)
            print('conv GPU time in one step: %.2f ms' % (tot / 1e3))
            for e in rows[:60]:
                print('%9.3f ms %4d  %-22s %s' % (e.device_time_total / 1e3, e.count, e.key[6:],
                                                  str(e.input_shapes)[:150]))
        sys.stdout.flush()

    def barrier():
        if world > 1:
            dist.barrier()
        if on_gpu:
            torch.cuda.synchronize()

    barrier()
    if args.profile_phases:
        trainer._reset_speed_accumulators()
    if args.verbose:
        try:  # phase marker for scripts/gpu/summarize_kernels.py (steady-state split)
            from imaginaire_amd.ops import _ext
            _ext.ext().profile_marker(1)
        except Exception:  # noqa: BLE001
            pass
    t0 = time.perf_counter()
    for it in range(args.steps):
        step(args.warmup + it)
        if rank == 0 and args.verbose:
            print('[bench] step {} queued'.format(it), flush=True)
    barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=device if args.backend == 'nccl' and on_gpu else 'cpu',
                     dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    if args.profile_phases and rank == 0:
        n = args.steps
        for k in ('gen_forw', 'gen_loss', 'gen_back', 'gen_step', 'gen_avg', 'dis_forw',
                  'dis_loss', 'dis_back', 'dis_step'):
            print('[bench] phase %-9s %8.1f ms/step' % (
                k, getattr(trainer, 'accu_%s_iter_time' % k) / n * 1e3), flush=True)
    # correctness of what was timed: the last step's losses (every rank) and, at world > 1,
    # whether the replicas still hold bitwise identical parameters (a rank-divergent replay or
    # unused-parameter mask would desynchronise them silently)
    losses = _last_losses(trainer)
    finite = all(v == v and abs(v) != float('inf') for v in losses.values())
    if world > 1:
        fl = torch.tensor([0.0 if finite else 1.0], dtype=torch.float64,
                          device=device if args.backend == 'nccl' and on_gpu else 'cpu')
        dist.all_reduce(fl, op=dist.ReduceOp.MAX)
        finite = float(fl.item()) == 0.0
    in_sync = _replicas_in_sync(trainer, world, device if args.backend == 'nccl' and on_gpu
                                else torch.device('cpu'))
    ms_per_step = elapsed / args.steps * 1e3
    value = world * bs * args.steps / elapsed
    mem_gb = torch.cuda.max_memory_allocated(device) / 2 ** 30 if on_gpu else 0.0
    sys.stdout = real_stdout
    if rank == 0:
        out = {
            'metric': 'imgs/sec (whole node) SPADE 256x512 training',
            'value': round(value, 3),
            'unit': 'images/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(ms_per_step, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': round(value / BASELINE_IMG_S, 3),
            'dtype': 'bf16' if on_gpu else 'fp32',
            'data': 'synthetic (COCO-Stuff-shaped: 183 classes + dont-care + edge), random-init weights',
            'config': {'model': 'SPADE/GauGAN (cocostuff base128_bs4 recipe: F=128, style VAE, '
                                'sync-BN SPADE 5x5 separate-projection, 2xPatchGAN+FPSE D, '
                                'VGG19 perceptual, EMA)',
                       'global_batch': bs * world, 'seq_len': None, 'resolution': '256x512',
                       'parallelism': 'dp%d' % world + ('-forced-dist' if args.force_dist else ''),
                       'kernels': 'eager-reference' if args.eager else 'hip',
                       'hipgraph': bool(graphed is not None and graphed.graph is not None),
                       'backend': args.backend if (world > 1 and on_gpu) else
                       ('gloo' if world > 1 else None),
                       'device': args.device},
            'peak_mem_gb_rank0': round(mem_gb, 2),
            'losses_rank0': losses,
            'losses_finite': finite,
            'replicas_in_sync': in_sync,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if not finite:
        print('[bench] NON-FINITE losses after the timed steps: %s' % json.dumps(losses),
              file=sys.stderr, flush=True)
        sys.exit(3)
    if in_sync is False:
        print('[bench] replicas hold different parameters after the timed steps',
              file=sys.stderr, flush=True)
        sys.exit(4)


def _last_losses(trainer):
    """The last step's D and G losses (graph outputs after a replay) as floats."""
    import torch
    out = {}
    for tag, src in (('G', getattr(trainer, 'gen_losses', {})),
                     ('D', getattr(trainer, 'dis_losses', {}))):
        for k, v in src.items():
            if torch.is_tensor(v) and v.numel() == 1:
                out['%s/%s' % (tag, k)] = round(float(v), 5)
    return out


def _replicas_in_sync(trainer, world, device):
    """World > 1: True when every rank holds bitwise identical G and D parameters (one fp64
    checksum per tensor of the fp32 bits, compared by a MIN / MAX all-reduce); None at world 1."""
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    sums = []
    for net in (trainer.net_G, trainer.net_D):
        if net is None:
            continue
        for p in net.parameters():
            # the int32 view makes the checksum sensitive to every bit of every element
            bits = p.detach().float().contiguous().view(torch.int32)
            sums.append(bits.to(torch.float64).sum() + 1e-3 * bits[::7].to(torch.float64).sum())
    v = torch.stack(sums).to(device)
    hi, lo = v.clone(), v.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    return bool(torch.equal(hi, lo))


if __name__ == '__main__':
    main()
