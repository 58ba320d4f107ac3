"""Multi-process data parallel (gloo, world size 2) on CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ddp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from imaginaire_amd.parallel import DistributedDataParallel
    torch.manual_seed(100 + rank)  # different init per rank: DDP must broadcast rank 0's
    net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    ddp = DistributedDataParallel(net, bucket_cap_mb=0.0005, first_bucket_mb=0.0001)
    assert len(ddp.buckets) > 1
    x = torch.randn(5, 8, generator=torch.Generator().manual_seed(rank))
    ddp.begin()
    loss = ddp(x).pow(2).sum()
    loss.backward()
    ddp.finish()
    grads = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
    params = torch.cat([p.detach().reshape(-1) for p in net.parameters()])
    q.put((rank, grads.numpy(), params.numpy(), x.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_gradients_are_averaged():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    import numpy as np
    g0, g1 = res[0][1], res[1][1]
    assert np.allclose(g0, g1, atol=1e-6)
    assert np.allclose(res[0][2], res[1][2])  # params broadcast from rank 0
    # reference: average of per-rank grads computed with rank-0 params
    torch.manual_seed(100)
    net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    gs = []
    for r in range(2):
        net.zero_grad()
        net(torch.from_numpy(res[r][3])).pow(2).sum().backward()
        gs.append(torch.cat([p.grad.reshape(-1) for p in net.parameters()]))
    avg = ((gs[0] + gs[1]) / 2).numpy()
    assert np.allclose(g0, avg, atol=1e-5)


def _syncbn_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from imaginaire_amd.layers.activation_norm import SyncBatchNorm
    torch.manual_seed(0)
    x_all = torch.randn(4, 6, 5, 5)
    x = x_all[rank * 2:(rank + 1) * 2].clone().requires_grad_(True)
    bn = SyncBatchNorm(6)
    y = bn(x, act_slope=0.2)
    (y * torch.arange(6.).view(1, 6, 1, 1)).sum().backward()
    q.put((rank, y.detach().numpy(), x.grad.numpy(), bn.running_mean.numpy(),
           bn.weight.grad.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_syncbn_matches_global_batchnorm():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_syncbn_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    import numpy as np
    torch.manual_seed(0)
    x_all = torch.randn(4, 6, 5, 5).requires_grad_(True)
    bn = torch.nn.BatchNorm2d(6)
    y = torch.nn.functional.leaky_relu(bn(x_all), 0.2)
    (y * torch.arange(6.).view(1, 6, 1, 1)).sum().backward()
    y_ref = y.detach().numpy()
    assert np.allclose(np.concatenate([res[0][1], res[1][1]]), y_ref, atol=1e-5)
    assert np.allclose(np.concatenate([res[0][2], res[1][2]]), x_all.grad.numpy(), atol=1e-4)
    assert np.allclose(res[0][3], bn.running_mean.detach().numpy(), atol=1e-6)
    # weight grad is local per rank (DDP averages it); sum over ranks == global
    assert np.allclose(res[0][4] + res[1][4], bn.weight.grad.numpy(), atol=1e-4)


def test_train_py_two_ranks_gloo(tmp_path):
    """train.py under torch.distributed.run with 2 gloo ranks: the whole trainer path
    (ModelAverage + native DDP + SyncBN groups + batched SN) on the SPADE unit config."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS='2')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), 'train.py',
           '--config', 'configs/unit_test/spade.yaml', '--backend', 'gloo',
           '--logdir', str(tmp_path)]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert 'Done with training' in r.stdout


def _unused_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from imaginaire_amd.optimizers import FusedAdam
    from imaginaire_amd.parallel import DistributedDataParallel
    torch.manual_seed(0)
    used = torch.nn.Linear(4, 4)
    unused = torch.nn.Linear(4, 4)
    net = torch.nn.ModuleDict({'used': used, 'unused': unused})
    res = {}
    for mode in ('local', 'global'):
        ddp = DistributedDataParallel(net, find_unused=mode)
        opt = FusedAdam(net.parameters(), lr=0.1)
        x = torch.randn(3, 4)
        # step 1: both branches used -> both get Adam moments
        ddp.begin()
        (used(x).sum() + unused(x).sum()).backward()
        ddp.finish()
        opt.step()
        opt.zero_grad(set_to_none=True)
        before = unused.weight.detach().clone()
        # step 2: the 'unused' branch gets no gradient -> grad None -> untouched by Adam
        ddp.begin()
        used(x).sum().backward()
        ddp.finish()
        res[mode] = (unused.weight.grad is None, used.weight.grad is not None)
        opt.step()
        res[mode] += (bool(torch.equal(before, unused.weight.detach())),)
        for h in ddp._hooks:
            h.remove()
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def _rank_skip_worker(rank, world, port, q):
    """Rank 1 skips a branch that rank 0 uses (data-dependent control flow, e.g. the
    vid2vid hand discriminator on a batch without hand pixels)."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from imaginaire_amd.optimizers import FusedAdam
    from imaginaire_amd.parallel import DistributedDataParallel
    torch.manual_seed(0)
    trunk = torch.nn.Linear(4, 4)
    hand = torch.nn.Linear(4, 4)
    never = torch.nn.Linear(4, 4)
    net = torch.nn.ModuleDict({'trunk': trunk, 'hand': hand, 'never': never})
    ddp = DistributedDataParallel(net)  # default: find_unused='global'
    opt = FusedAdam(net.parameters(), lr=0.1)
    grads = []
    for it in range(3):
        x = torch.randn(3, 4, generator=torch.Generator().manual_seed(10 * it + rank))
        ddp.begin()
        loss = trunk(x).sum()
        if rank == 0 or it == 0:
            loss = loss + hand(x).pow(2).sum()
        loss.backward()
        ddp.finish()
        grads.append((hand.weight.grad is None, never.weight.grad is None,
                      None if hand.weight.grad is None else hand.weight.grad.clone().numpy()))
        opt.step()
        opt.zero_grad(set_to_none=True)
    params = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).numpy()
    q.put((rank, params, grads))
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_rank_dependent_skip_keeps_replicas_identical():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_skip_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    import numpy as np
    (_, p0, g0), (_, p1, g1) = res
    assert np.array_equal(p0, p1), 'replicas diverged after a rank-local skip'
    for it in range(3):
        # the branch rank 1 skipped still carries the averaged gradient on rank 1
        assert g0[it][0] is False and g1[it][0] is False
        assert np.allclose(g0[it][2], g1[it][2])
        # a branch no rank used keeps grad None everywhere
        assert g0[it][1] is True and g1[it][1] is True


def test_ddp_unused_parameters_keep_grad_none():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_unused_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for _, r in res:
        for mode in ('local', 'global'):
            assert r[mode] == (True, True, True), (mode, r[mode])


def _agree_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from imaginaire_amd.ops.conv import _agree
    # rank-local timings disagree on which candidate is faster; the summed ones decide
    times = {('w', (1, 2)): {'k11': 1.0 + 3 * rank, 'miopen': 2.0},
             ('d', (3,)): {'k10s': 5.0 - 4 * rank, 'miopen': 3.0}}
    out = _agree(times)
    q.put((rank, {k: min(v, key=v.get) for k, v in out.items()}))
    dist.barrier()
    dist.destroy_process_group()


def test_kernel_choice_agreed_across_ranks():
    """Per-shape autotune results (k11 vs MIOpen wgrad, k10 phases vs MIOpen deconv) are summed
    over ranks before the argmin, so every rank runs the same kernel."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1]
    assert res[0][1][('w', (1, 2))] == 'miopen'  # 1+4 > 2+2
    assert res[0][1][('d', (3,))] == 'k10s'      # 5+1 = 6 == 3+3 -> min picks first (k10s)


def _capture_agree_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from imaginaire_amd.utils.cuda_graph import agree_capture
    out = {
        'both_ok': agree_capture(True, 1234),
        'one_failed': agree_capture(rank == 0, 1234),     # rank 1's capture raised
        'sig_differs': agree_capture(True, 1234 + rank),  # ranks captured different batches
        'none_ok': agree_capture(False, 7),
    }
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_capture_outcome_agreed_across_ranks():
    """Multi-rank hipGraph capture (utils/cuda_graph.py): every rank keeps its graph only if
    every rank captured the same batch structure; one failed or different capture sends all
    ranks to the eager step together."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_capture_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for _, r in res:
        assert r == {'both_ok': True, 'one_failed': False, 'sig_differs': False,
                     'none_ok': False}, r


def _pending_union_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from imaginaire_amd.ops import conv
    # iteration 1: nothing pending anywhere -> both ranks still run the count exchange
    first = conv._pending_union()
    # iteration 2: only rank 1 saw a new weight-gradient shape (e.g. a per-rank hand crop)
    if rank == 1:
        key = ((2, 64, 8, 8), (2, 64, 8, 8), (64, 64, 3, 3), (1, 1), (1, 1), (1, 1), 64, 64,
               torch.bfloat16)
        conv._WGRAD_PENDING[key] = (torch.bfloat16, torch.bfloat16, torch.bfloat16)
    second = conv._pending_union()
    q.put((rank, first, [(k, key[0]) for k, key, _ in second]))
    dist.barrier()
    dist.destroy_process_group()


def test_tune_pending_union_when_one_rank_has_keys():
    """a rank with no pending kernel-choice keys must not skip the exchange a rank
    with new keys enters; both ranks see the same union (and would time the same shapes)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pending_union_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0][1] == [] and res[1][1] == []
    assert res[0][2] == res[1][2] == [('w', (2, 64, 8, 8))]


def test_video_family_rank_uniform_follows_config():
    """the vid2vid family declares rank-uniform control flow per config — the
    street / face recipes (no additional discriminators) get DDP's rank-local unused mask (no
    host sync per per-frame backward, capturable at world > 1); the pose recipes' hand / face
    discriminators keep the global mask; wc-vid2vid stays global."""
    from imaginaire_amd.config import Config
    from imaginaire_amd.utils.trainer import _find_unused_mode
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    want = {'vid2vid_street': 'local', 'fs_vid2vid_face': 'local', 'vid2vid_pose': 'global',
            'fs_vid2vid_pose': 'global', 'wc_vid2vid': 'global', 'spade': 'local'}
    for name, mode in want.items():
        cfg = Config(os.path.join(root, 'configs', 'unit_test', name + '.yaml'))
        assert _find_unused_mode(cfg) == mode, name


def _video_local_worker(rank, world, port, q, tmp):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from torch.utils.data import default_collate
    from imaginaire_amd.config import Config
    from imaginaire_amd.datasets.synthetic import Dataset
    from imaginaire_amd.parallel import DistributedDataParallel
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = Config(os.path.join(root, 'configs', 'unit_test', 'vid2vid_street.yaml'))
    cfg.logdir = tmp
    cfg.data.train.initial_sequence_length = 2
    cfg.data.train.max_sequence_length = 2
    ds = Dataset(cfg)

    class _Loader(list):
        dataset = ds

    torch.manual_seed(0)
    nets = get_model_optimizer_and_scheduler(cfg, seed=0)
    tr = get_trainer(cfg, *nets, train_data_loader=_Loader(), val_data_loader=None)
    tr.init_temporal_network()
    ds.set_sequence_length(2)
    tr.sequence_length = 2
    assert isinstance(tr.net_G, DistributedDataParallel) or \
        isinstance(getattr(tr.net_G, 'module', None), DistributedDataParallel) or \
        any(isinstance(m, DistributedDataParallel) for m in tr.net_G.modules())
    ddps = [m for n in (tr.net_G, tr.net_D) for m in [n] + list(n.modules())
            if isinstance(m, DistributedDataParallel)]
    modes = sorted({m.find_unused for m in ddps})
    bs = cfg.data.train.batch_size
    # each rank trains on its own samples
    data = default_collate([ds[(rank * bs + j) % len(ds)] for j in range(bs)])
    data = tr.start_of_iteration(data, 0)
    tr.dis_update(data)
    tr.gen_update(data)
    losses = [float(v) for v in tr.gen_losses.values()]
    params = torch.cat([p.detach().reshape(-1) for n in (tr.net_G, tr.net_D)
                        for p in n.parameters()])
    q.put((rank, modes, params.numpy(), losses))
    dist.barrier()
    dist.destroy_process_group()


def test_video_family_local_mask_keeps_replicas_identical(tmp_path):
    """2 gloo ranks, vid2vid street unit config, different data per rank, the rank-local unused
    mask: after a whole per-frame D / G sequence update every rank holds identical G and D
    parameters (the mask agreed by construction: the same sub-networks ran everywhere)."""
    import numpy as np
    world = 2
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_video_local_worker, args=(r, world, port, q, str(tmp_path)))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r = q.get(timeout=540)
            res[r[0]] = r[1:]
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    assert res[0][0] == ['local'], res[0][0]
    assert all(np.isfinite(v) for v in res[0][2] + res[1][2])
    assert res[0][2] != res[1][2], 'ranks trained on the same data'
    assert np.array_equal(res[0][1], res[1][1]), 'replicas diverged'
