"""The bench's multi-rank step on the GPU: two processes on
cuda:0, each solving its contiguous shard through the C ABI into the slots of
hmpc_dist.ResultExchange (side-stream all-gather pipelined with the next
solve, double-buffered), over gloo with CUDA tensors -- the one-GPU box cannot
run two RCCL ranks.  After three steps every rank must hold exactly the
single-process objectives and statuses of the whole batch, in rank order."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PER_RANK = 1024
N = 10
STEPS = 3


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ctx(hmpc):
    from oracle import hmpc_oracle as ho
    c = ho.runner_constants()
    return hmpc.Context('3f', N, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])


def _inputs(start, count, dev):
    import hmpc_plan
    inst = hmpc_plan.sample_instances(count, N, curve=True, seed=5, mu_sweep=(0.3, 1.2),
                                      start=start)
    return {k: torch.from_numpy(np.ascontiguousarray(inst[k])).to(dev)
            for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}


def _worker(rank, world, port, q):
    import sys
    for p in (os.path.join(ROOT, 'hopper-mpc-inertial_amd'), ROOT):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import hmpc
    import hmpc_dist
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    d = _inputs(hmpc_dist.shard_start(rank, PER_RANK), PER_RANK, dev)
    ctx = _ctx(hmpc)
    u = torch.empty((PER_RANK, N, 6), dtype=torch.float64, device=dev)
    ex = hmpc_dist.ResultExchange(PER_RANK, dev)
    slot = None
    for _ in range(STEPS):
        ob, sb = ex.outputs()
        ctx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'],
                         out=dict(u=u, obj=ob, status=sb))
        slot = ex.exchange()
    ex.wait()
    torch.cuda.synchronize(dev)
    oa, sa = ex.results(slot)
    q.put((rank, oa.cpu().numpy().copy(), sa.cpu().numpy().copy()))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


def test_pipelined_exchange_equals_single_process():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X')
    import hmpc
    d = _inputs(0, PER_RANK * world, torch.device('cuda', 0))
    ctx1 = _ctx(hmpc)
    out = ctx1.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
    torch.cuda.synchronize()
    obj_ref, st_ref = out['obj'].cpu().numpy(), out['status'].cpu().numpy()
    ctx1.close()
    assert (st_ref == 0).mean() > 0.9
    for _, oa, sa in res:
        assert np.array_equal(sa, st_ref)
        assert np.array_equal(oa, obj_ref)   # bitwise: shards are batch-position invariant
