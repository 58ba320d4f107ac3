"""Multi-rank correctness of the HIP SyncBN and the bucketed DDP on the GPU.

Two ranks share the one GPU of the test box (gloo process group; RCCL cannot place two ranks
on one device). Reference semantics:
  * SyncBN: torch.nn.SyncBatchNorm (reference layers/activation_norm.py:403-410) — the
    sync_batch fused norm on per-rank halves must equal batch norm over the concatenated batch;
  * DDP: torch DDP (reference utils/trainer.py:206-214) — gradients after backward equal the
    single-process gradients of the whole batch (mean losses, SyncBN statistics), on both the
    fp32 and the bf16 wire.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    import faulthandler
    import sys
    import torch.distributed as dist
    # a hung collective must end the child (and print where) well inside the box's 180 s
    # silence limit: the parent then sees a non-zero exit code instead of waiting
    faulthandler.dump_traceback_later(150, exit=True, file=sys.__stderr__)
    print('[dist-test] rank %d starting' % rank, file=sys.__stderr__, flush=True)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    print('[dist-test] rank %d joined the gloo group' % rank, file=sys.__stderr__, flush=True)
    return dist


def _to_np(obj):
    if torch.is_tensor(obj):
        return ('__tensor__', obj.detach().cpu().numpy())
    if isinstance(obj, dict):
        return {k: _to_np(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_np(o) for o in obj)
    return obj


def _to_torch(obj):
    if isinstance(obj, tuple) and len(obj) == 2 and isinstance(obj[0], str) and \
            obj[0] == '__tensor__':
        return torch.from_numpy(obj[1])
    if isinstance(obj, dict):
        return {k: _to_torch(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_torch(o) for o in obj)
    return obj


class _NpQueue:
    """Results travel as numpy arrays: a CPU tensor put on a multiprocessing queue is shared
    through a file descriptor served by the SENDING process, which may already have exited
    when the parent unpickles it (FileNotFoundError on the resource-sharer socket)."""

    def __init__(self, q):
        self.q = q

    def put(self, obj):
        self.q.put(_to_np(obj))

    def get(self, timeout=None):
        return _to_torch(self.q.get(timeout=timeout))


def _spawn(target, world, *args):
    ctx = mp.get_context('spawn')
    q = _NpQueue(ctx.Queue())
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=170) for _ in range(world)], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return res


def _bn_inputs(dtype):
    g = torch.Generator().manual_seed(0)
    N, C, H, W = 4, 64, 8, 12
    x = torch.randn(N, C, H, W, generator=g) * 2 + 0.5
    gb = torch.randn(N, 2 * C, H, W, generator=g) * 0.3
    gout = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, generator=g) * 0.5 + 1
    b = torch.randn(C, generator=g) * 0.1
    return x.to(dtype), gb.to(dtype), gout, w, b


def _syncbn_worker(rank, world, port, q, dtype):
    dist = _init(rank, world, port)
    from imaginaire_amd.ops.norm import fused_norm_act
    x, gb, gout, w, b = _bn_inputs(dtype)
    n = x.shape[0] // world
    sl = slice(rank * n, (rank + 1) * n)
    cl = torch.channels_last
    xr = x[sl].cuda().contiguous(memory_format=cl).requires_grad_(True)
    gbr = gb[sl].cuda().contiguous(memory_format=cl).requires_grad_(True)
    wr = w.cuda().requires_grad_(True)
    br = b.cuda().requires_grad_(True)
    rm = torch.zeros(x.shape[1], device='cuda')
    rv = torch.ones(x.shape[1], device='cuda')
    y = fused_norm_act(xr, 'sync_batch', wr, br, gb=gbr, running_mean=rm, running_var=rv,
                       training=True, momentum=0.1, slope=0.2)
    y.backward(gout[sl].cuda().to(y.dtype).contiguous(memory_format=cl))
    torch.cuda.synchronize()
    q.put((rank, y.detach().float().cpu(), xr.grad.float().cpu(), gbr.grad.float().cpu(),
           wr.grad.cpu(), br.grad.cpu(), rm.cpu(), rv.cpu()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_hip_syncbn_world2_matches_full_batch(dtype):
    res = _spawn(_syncbn_worker, 2, dtype)
    x, gb, gout, w, b = _bn_inputs(dtype)
    C = x.shape[1]
    xr = x.float().requires_grad_(True)
    gbr = gb.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    rm, rv = torch.zeros(C), torch.ones(C)
    yr = F.batch_norm(xr, rm, rv, wr, br, True, 0.1, 1e-5)
    yr = F.leaky_relu(yr * (1 + gbr[:, :C]) + gbr[:, C:], 0.2)
    yr.backward(gout)
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    y = torch.cat([r[1] for r in res])
    dx = torch.cat([r[2] for r in res])
    dgb = torch.cat([r[3] for r in res])
    assert torch.allclose(y, yr, atol=tol * 4, rtol=tol), (y - yr).abs().max()
    sc = float(xr.grad.abs().max())
    assert torch.allclose(dx, xr.grad, atol=tol * 4 * sc, rtol=tol * 4), (dx - xr.grad).abs().max()
    assert torch.allclose(dgb, gbr.grad, atol=tol * 4, rtol=tol * 4)
    # per-rank affine gradients are partial sums over the rank's pixels (DDP averages them)
    dw = res[0][4] + res[1][4]
    db = res[0][5] + res[1][5]
    assert torch.allclose(dw, wr.grad, atol=tol * 20, rtol=tol * 4), (dw - wr.grad).abs().max()
    assert torch.allclose(db, br.grad, atol=tol * 20, rtol=tol * 4)
    for r in res:  # running statistics of the GLOBAL batch on every rank
        assert torch.allclose(r[6], rm, atol=1e-4, rtol=1e-3)
        assert torch.allclose(r[7], rv, atol=1e-4, rtol=1e-3)


def _spade_norm_worker(rank, world, port, q):
    """One SPADE norm layer (sync-BN, separate γ / β projections) on this rank's half batch."""
    if world > 1:
        dist = _init(rank, world, port)
    else:
        import faulthandler
        import sys
        faulthandler.dump_traceback_later(150, exit=True, file=sys.__stderr__)
        torch.cuda.set_device(0)
    from types import SimpleNamespace as NS
    from imaginaire_amd.layers.activation_norm import SpatiallyAdaptiveNorm
    from imaginaire_amd.ops.norm import DeferredSyncBwd
    torch.manual_seed(3)
    layer = SpatiallyAdaptiveNorm(64, 8, num_filters=32, kernel_size=3, separate_projection=True,
                                  activation_norm_type='sync_batch',
                                  activation_norm_params=NS(affine=False)).cuda()
    layer = layer.to(memory_format=torch.channels_last)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(4, 64, 16, 24, generator=g) * 1.5 + 0.3
    lab = torch.randn(4, 8, 16, 24, generator=g)
    gout = torch.randn(4, 64, 16, 24, generator=g)
    n = 4 // world
    sl = slice(rank * n, (rank + 1) * n)
    cl = torch.channels_last
    xr = x[sl].cuda().contiguous(memory_format=cl).requires_grad_(True)
    y = layer(xr, lab[sl].cuda().contiguous(memory_format=cl), act_slope=0.2)
    y.backward(gout[sl].cuda().contiguous(memory_format=cl))
    torch.cuda.synchronize()
    # numpy, not torch tensors: a queued CPU tensor travels as a shared-memory fd that dies
    # with this process (the world-1 reference exits right after the put)
    grads = {k: p.grad.detach().float().cpu().numpy() for k, p in layer.named_parameters()
             if p.grad is not None}
    q.put((rank, y.detach().float().cpu().numpy(), xr.grad.float().cpu().numpy(), grads,
           DeferredSyncBwd.completed))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def test_spade_syncbn_async_backward_world2():
    """The SPADE norm's deferred sync-BN data gradient (all-reduce overlapped with the γ|β /
    mlp convolution backward, finished by the join node) == the full batch on one process."""
    res = _spawn(_spade_norm_worker, 2)
    ref = _spawn(_spade_norm_worker, 1)[0]
    assert all(r[4] >= 1 for r in res), 'the deferred (async) sync-BN backward did not run'
    T = torch.from_numpy
    y = torch.cat([T(r[1]) for r in res])
    dx = torch.cat([T(r[2]) for r in res])
    torch.testing.assert_close(y, T(ref[1]), atol=2e-4, rtol=1e-3)
    torch.testing.assert_close(dx, T(ref[2]), atol=2e-4 * float(abs(ref[2]).max()), rtol=1e-3)
    for k, gr in ref[3].items():  # per-rank weight grads are partial sums of the batch loss
        gr = T(gr)
        gs = T(res[0][3][k]) + T(res[1][3][k])
        torch.testing.assert_close(gs, gr, atol=1e-3 * float(gr.abs().max()) + 1e-5, rtol=2e-3,
                                   msg=k)


def _spade_grads(rank, world, comm):
    """G gradients of one SPADE G update (fp32, HIP path), rank's half of a 2-sample batch."""
    from imaginaire_amd.config import Config
    from imaginaire_amd.datasets.synthetic import DeviceBatchSource
    from imaginaire_amd.utils.trainer import get_model_optimizer_and_scheduler, get_trainer
    cfg = Config(os.path.join(ROOT, 'configs', 'unit_test', 'spade.yaml'))
    cfg.logdir = '/tmp/iamd_ddp_test_%d' % rank
    cfg.speed_benchmark = False
    cfg.trainer.amp = 'O0'
    cfg.trainer.model_average = False
    cfg.trainer.ddp_bucket_mb = 1  # many buckets: exercises the per-bucket launch order
    if comm:
        cfg.trainer.ddp_comm_dtype = comm
    nets = get_model_optimizer_and_scheduler(cfg, seed=0)
    tr = get_trainer(cfg, *nets, train_data_loader=[], val_data_loader=None)
    enc = tr.net_G_module.style_encoder
    enc.freeze_random = True
    style_dims = cfg.gen.style_dims
    eps = torch.randn(2, style_dims, generator=torch.Generator().manual_seed(5)).cuda()
    src = DeviceBatchSource(cfg, 2, torch.device('cuda', 0), pool=1, seed=0)
    data = src.next()
    n = 2 // world
    sl = slice(rank * n, (rank + 1) * n)
    data = {k: (v[sl].clone() if torch.is_tensor(v) and v.dim() > 0 and v.shape[0] == 2 else v)
            for k, v in data.items()}
    enc.eps = eps[sl]
    data = tr.start_of_iteration(data, 0)
    tr.gen_update(data)
    torch.cuda.synchronize()
    names, grads = [], []
    for name, p in tr.net_G_module.named_parameters():
        if p.grad is not None:
            names.append(name)
            grads.append(p.grad.detach().float().reshape(-1).cpu())
    return names, torch.cat(grads)


def _ddp_worker(rank, world, port, q, comm):
    dist = _init(rank, world, port)
    names, g = _spade_grads(rank, world, comm)
    q.put((rank, names, g))
    dist.barrier()
    dist.destroy_process_group()


def _ref_worker(rank, world, port, q):
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(150, exit=True, file=sys.__stderr__)
    torch.cuda.set_device(0)
    names, g = _spade_grads(0, 1, None)
    q.put((0, names, g))


@pytest.mark.parametrize('comm', [None, 'bf16'])
def test_ddp_spade_world2_grads_match_single_process(comm):
    res = _spawn(_ddp_worker, 2, comm)
    ref = _spawn(_ref_worker, 1)[0]
    (_, n0, g0), (_, n1, g1) = res
    assert n0 == n1 == ref[1], 'different parameter sets received gradients'
    # both ranks hold the same (averaged) gradient
    assert torch.equal(g0, g1)
    gr = ref[2]
    rel = float((g0 - gr).norm() / gr.norm())
    # fp32 runs land at 1.5e-3 .. 2.05e-3 (the batch statistics reduce in a different order on
    # two ranks, and the D / VGG reductions use atomics): 3e-3 leaves room for that spread
    assert rel < (2e-2 if comm else 3e-3), rel


def _rccl_world1_worker(rank, world, port, q):
    import sys
    import faulthandler
    import torch.distributed as dist
    faulthandler.dump_traceback_later(150, exit=True, file=sys.__stderr__)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK='0', WORLD_SIZE='1',
                      LOCAL_RANK='0')
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
    from imaginaire_amd.parallel import DistributedDataParallel
    out = {}
    for comm in (None, torch.bfloat16):
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Conv2d(8, 16, 3, padding=1), torch.nn.ReLU(),
                                  torch.nn.Conv2d(16, 4, 3, padding=1)).cuda()
        unused = torch.nn.Linear(3, 3).cuda()
        holder = torch.nn.ModuleDict({'net': net, 'unused': unused})
        ref = [p.detach().clone() for p in net.parameters()]
        ddp = DistributedDataParallel(holder, bucket_cap_mb=0.002, first_bucket_mb=0.001,
                                      comm_dtype=comm, _force_distributed=True)
        x = torch.randn(2, 8, 12, 12, device='cuda')
        grads = []
        for it in range(2):  # the second backward must not see the first one's gradients
            ddp.begin()
            ddp.module['net'](x * (it + 1)).pow(2).mean().backward()
            ddp.finish()
            grads.append([p.grad.detach().clone() for p in net.parameters()])
        # plain single-process gradients of the same two backwards
        plain = torch.nn.Sequential(torch.nn.Conv2d(8, 16, 3, padding=1), torch.nn.ReLU(),
                                    torch.nn.Conv2d(16, 4, 3, padding=1)).cuda()
        with torch.no_grad():
            for p, r in zip(plain.parameters(), ref):
                p.copy_(r)
        ok = True
        for it in range(2):
            plain.zero_grad(set_to_none=True)
            plain(x * (it + 1)).pow(2).mean().backward()
            tol = 1e-5 if comm is None else 1e-2
            for g, p in zip(grads[it], plain.parameters()):
                ok &= bool(torch.allclose(g, p.grad, atol=tol, rtol=tol))
        ok &= all(p.grad is None for p in unused.parameters())
        ok &= len(ddp.buckets) > 1
        out['bf16' if comm else 'fp32'] = (ok, ddp._avg)
    q.put((rank, out))
    dist.destroy_process_group()


def _zero_copy_worker(rank, world, port, q):
    import sys
    import faulthandler
    import torch.distributed as dist
    faulthandler.dump_traceback_later(150, exit=True, file=sys.__stderr__)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK='0', WORLD_SIZE='1',
                      LOCAL_RANK='0')
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
    from imaginaire_amd.parallel import DistributedDataParallel
    from imaginaire_amd.ops import conv as C
    C._MFMA_MIN_BLOCKS = 0
    cl = torch.channels_last

    from imaginaire_amd.layers.spectral_norm import _SNScale
    gen = torch.Generator(device='cuda').manual_seed(3)
    su = torch.nn.functional.normalize(torch.randn(128, device='cuda', generator=gen), dim=0)
    sv = torch.nn.functional.normalize(torch.randn(128 * 9, device='cuda', generator=gen), dim=0)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Conv2d(64, 128, 3, padding=1)
            self.b = torch.nn.Conv2d(128, 128, 3, padding=1)  # used twice per forward
            self.g = torch.nn.Parameter(torch.ones(128))       # not a conv weight: copied
            # materialised spectral norm (the SPADE gamma|beta path): the SN backward writes
            # dW into the bucket (sn_scale_backward dst)
            self.s = torch.nn.Conv2d(128, 128, 3, padding=1, bias=False)

        def forward(self, x):
            h = C.conv2d_act(x, self.a.weight, self.a.bias, 1, 1, 1, 0.2)
            h = C.conv2d(h, self.b.weight, self.b.bias, 1, 1) * self.g.view(1, -1, 1, 1)
            with torch.autocast('cuda', enabled=False):  # (fp32 sigma, as the SN group's)
                sigma = su @ self.s.weight.detach().reshape(128, -1) @ sv
                ws = _SNScale.apply(self.s.weight, su, sv, sigma.reshape(1))
            h = C.conv2d(h, ws.to(torch.bfloat16), None, 1, 1)
            return C.conv2d(h, self.b.weight, None, 1, 1)

    torch.manual_seed(0)
    net = Net().cuda().to(memory_format=cl)
    ref = Net().cuda().to(memory_format=cl)
    ref.load_state_dict(net.state_dict())
    ddp = DistributedDataParallel(net, _force_distributed=True)
    x = torch.randn(2, 64, 16, 64, device='cuda').contiguous(memory_format=cl)
    out = {}
    for it in range(2):
        ddp.begin()
        with torch.autocast('cuda', dtype=torch.bfloat16):
            y = net(x * (it + 1))
        y.float().pow(2).mean().backward()
        ddp.finish()
        ref.zero_grad(set_to_none=True)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            yr = ref(x * (it + 1))
        yr.float().pow(2).mean().backward()
        ok = True
        for (n, p), pr in zip(net.named_parameters(), ref.parameters()):
            bi, off = ddp._param_bucket[p]
            view_ptr = ddp.buckets[bi].flat[off:].data_ptr()
            ok &= p.grad.data_ptr() == view_ptr
            ok &= bool(torch.allclose(p.grad, pr.grad, atol=1e-4, rtol=1e-3))
        out[it] = ok
    # copied by the hook: a.bias, b.bias, g, and b.weight (its two uses are summed by autograd,
    # the first into the bucket) at most; a.weight lands in the bucket directly
    out['copies'] = ddp.n_copies
    q.put((rank, out))
    dist.destroy_process_group()


def test_ddp_zero_copy_weight_gradients_world1():
    """k11 writes conv weight gradients straight into the DDP bucket (ops/conv.py
    _take_grad_dest): the parameter's .grad IS its bucket slice, the hook copies only the other
    gradients, and the values equal the plain (undistributed) backward, including a weight used
    twice in one backward."""
    (_, out), = _spawn(_zero_copy_worker, 1)
    assert out[0] and out[1], out
    # per backward at most: a.bias, b.bias, g, b.weight -> 4; a.weight never (all five were
    # copied before round 6: 10 over the two backwards)
    assert out['copies'] <= 2 * 4, out


def test_ddp_rccl_world1_buckets_avg_and_unused():
    """The bucketed DDP on a real RCCL communicator (world size 1, forced through the
    distributed path): ReduceOp.AVG is detected, hook-filled buckets reproduce the plain
    gradients over two backwards (fp32 and bf16 wire), unused parameters keep grad None."""
    (_, out), = _spawn(_rccl_world1_worker, 1)
    for k, (ok, avg) in out.items():
        assert ok, k
        assert avg, 'RCCL should average in the collective (ReduceOp.AVG)'
