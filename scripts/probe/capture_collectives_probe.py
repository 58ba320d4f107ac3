"""Which torch.distributed (RCCL) call patterns survive hipGraph capture on this stack?

Each case runs in its own process on a world-1 RCCL group: warm up eagerly on a side stream,
capture, replay twice, check the result, and let the ProcessGroupNCCL watchdog poll for a
while (a work it polls whose event was recorded inside the capture aborts the process:
'operation not permitted on an event last recorded in a capturing stream')."""
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp


def _case(name, port, q, mode='global'):
    import faulthandler
    faulthandler.dump_traceback_later(60, exit=True)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK='0', WORLD_SIZE='1')
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
    x = torch.ones(1024, device='cuda', requires_grad=True)
    buf = torch.zeros(1024, device='cuda')
    out = torch.zeros(2, 1024, device='cuda')

    def body():
        if name == 'allreduce_sync':
            buf.copy_(x.detach() * 2)
            dist.all_reduce(buf)
        elif name == 'allreduce_async_wait':
            buf.copy_(x.detach() * 2)
            w = dist.all_reduce(buf, async_op=True)
            w.wait()
        elif name == 'allgather_tensor_async':
            w = dist.all_gather_into_tensor(out[:1], (x.detach() * 2).contiguous(), async_op=True)
            w.wait()
            buf.copy_(out[0])
        elif name == 'allreduce_in_backward_hook':
            works = []
            y = (x * 2)
            h = x.register_post_accumulate_grad_hook(
                lambda p: works.append(dist.all_reduce(p.grad, async_op=True)))
            x.grad = None
            y.sum().backward()
            h.remove()
            for w in works:
                w.wait()
            buf.copy_(x.grad)
        elif name.startswith('slow_'):
            # a long capture (like a whole training step): the watchdog polls meanwhile
            buf.copy_(x.detach() * 2)
            dist.all_reduce(buf, async_op=True).wait()
            if torch.cuda.is_current_stream_capturing():
                time.sleep(3)
        elif name == 'allreduce_in_autograd_fn':
            class F(torch.autograd.Function):
                @staticmethod
                def forward(ctx, a):
                    return a * 2

                @staticmethod
                def backward(ctx, g):
                    g = g.clone()
                    dist.all_reduce(g, async_op=True).wait()
                    return g * 2
            x.grad = None
            F.apply(x).sum().backward()
            buf.copy_(x.grad)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=s, capture_error_mode=mode):
            body()
        for _ in range(2):
            buf.zero_()
            g.replay()
        torch.cuda.synchronize()
        ok = float(buf[0]) == 2.0
        time.sleep(3)  # let the watchdog poll
        q.put((name + '/' + mode, 'ok' if ok else 'wrong value %s' % float(buf[0])))
    except Exception as e:  # noqa: BLE001
        q.put((name + '/' + mode, 'capture failed: %s' % str(e).splitlines()[0][:200]))
    dist.destroy_process_group()


def main():
    cases = [('allreduce_sync', 'global'), ('allreduce_async_wait', 'global'),
             ('allgather_tensor_async', 'global'), ('allreduce_in_backward_hook', 'global'),
             ('allreduce_in_autograd_fn', 'global'), ('slow_allreduce', 'global'),
             ('slow_allreduce', 'thread_local'), ('slow_allreduce', 'relaxed')]
    if len(sys.argv) > 1:
        cases = [c for c in cases if c[0] in sys.argv[1:]]
    ctx = mp.get_context('spawn')
    for c, mode in cases:
        s = socket.socket()
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
        s.close()
        q = ctx.Queue()
        p = ctx.Process(target=_case, args=(c, port, q, mode))
        p.start()
        try:
            res = q.get(timeout=90)
        except Exception:  # noqa: BLE001
            res = (c + '/' + mode, 'no result')
        p.join(20)
        if p.is_alive():
            p.kill()
        print('%-28s %-40s exit=%s' % (res[0], res[1], p.exitcode), flush=True)


if __name__ == '__main__':
    main()
