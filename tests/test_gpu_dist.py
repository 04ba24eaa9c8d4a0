"""The bench's multi-rank step on the GPU: two processes on
cuda:0, each solving its contiguous shard through the C ABI into the slots of
hmpc_dist.ResultExchange (side-stream all-gather pipelined with the next
solve, double-buffered), over gloo with CUDA tensors -- the one-GPU box cannot
run two RCCL ranks.  After three steps every rank must hold exactly the
single-process objectives and statuses of the whole batch, in rank order.

Two workloads: configs[2]'s weak split (N = 10, --curve, equal shards) and
configs[3]'s strong split (N = 20, straight plan, mu sweep, the Riccati
kernel; a global batch of 4097 that two ranks cannot split evenly, so the
exchange runs with padded slots), where every rank's u* must also equal the
single-process u* bit for bit."""
import os
import socket

import numpy as np
import pytest
from conftest import DENSE10_3F

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


# name -> (horizon, --curve, global batch or 0 = PER_RANK per rank, kernel)
WORKLOADS = {'cfg2_weak': (N, True, 0, DENSE10_3F),
             'cfg3_strong': (20, False, 4097, 'hmpc::ric_kernel<3, 2, 20, 38, 0>')}


def _ctx(hmpc, n=N):
    from oracle import hmpc_oracle as ho
    c = ho.runner_constants()
    return hmpc.Context('3f', n, t=c['t'], m=c['m'], g=c['g'], mu=1.0, Jinv=c['Jinv'], rh=c['rh'])


def _inputs(start, count, dev, n=N, curve=True):
    import hmpc_plan
    inst = hmpc_plan.sample_instances(count, n, curve=curve, seed=5, mu_sweep=(0.3, 1.2),
                                      start=start)
    return {k: torch.from_numpy(np.ascontiguousarray(inst[k])).to(dev)
            for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C', 'mu')}


def _worker(rank, world, port, q, wl, backend='gloo'):
    import sys
    for p in (os.path.join(ROOT, 'hopper-mpc-inertial_amd'), ROOT):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    if backend == 'nccl':
        dist.init_process_group('nccl', rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group('gloo', rank=rank, world_size=world)
    import hmpc
    import hmpc_dist
    n, curve, gb, kernel = WORKLOADS[wl]
    if gb:   # strong split of a fixed global batch (bench.py --global-batch)
        start, cnt = hmpc_dist.strong_shard(gb, world, rank)
        counts = [hmpc_dist.strong_shard(gb, world, r)[1] for r in range(world)]
    else:
        start, cnt, counts = hmpc_dist.shard_start(rank, PER_RANK), PER_RANK, None
    d = _inputs(start, cnt, dev, n, curve)
    ctx = _ctx(hmpc, n)
    assert ctx.kernel_name == kernel, ctx.kernel_name
    u = torch.empty((cnt, n, 6), dtype=torch.float64, device=dev)
    ex = hmpc_dist.ResultExchange(cnt, dev, counts=counts)
    slot = None
    for _ in range(STEPS):
        ob, sb = ex.outputs()
        ctx.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'],
                         out=dict(u=u, obj=ob, status=sb))
        slot = ex.exchange()
    ex.wait()
    torch.cuda.synchronize(dev)
    oa, sa = ex.results(slot)
    q.put((rank, oa.cpu().numpy().copy(), sa.cpu().numpy().copy(), start, u.cpu().numpy().copy(),
           dict(ex.calls), dist.get_backend()))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize('wl', list(WORKLOADS))
def test_pipelined_exchange_equals_single_process(wl):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, wl)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X')
    import hmpc
    n, curve, gb, _ = WORKLOADS[wl]
    total = gb or PER_RANK * world
    d = _inputs(0, total, torch.device('cuda', 0), n, curve)
    ctx1 = _ctx(hmpc, n)
    out = ctx1.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
    torch.cuda.synchronize()
    obj_ref, st_ref = out['obj'].cpu().numpy(), out['status'].cpu().numpy()
    u_ref = out['u'].cpu().numpy()
    ctx1.close()
    assert (st_ref == 0).mean() > 0.9
    for _, oa, sa, start, u, calls, backend in res:
        assert backend == 'gloo' and calls['all_gather_list'] == STEPS, calls
        assert np.array_equal(sa, st_ref)
        assert np.array_equal(oa, obj_ref)   # bitwise: shards are batch-position invariant
        assert np.array_equal(u, u_ref[start:start + len(u)])
    assert sorted(r[3] for r in res)[1] == len(min(res, key=lambda r: r[3])[4])   # shards tile


def test_rccl_exchange_one_rank():
    """The exchange's RCCL branch on hardware: one rank on the nccl (= RCCL)
    backend, so ResultExchange takes all_gather_into_tensor on its side
    stream (a one-GPU box cannot hold two RCCL ranks; the 2/4/8-rank
    collective is the driver's SCALE run).  The gathered objectives and
    statuses equal a plain solve of the same batch bit for bit."""
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), q, 'cfg2_weak', 'nccl'))
    p.start()
    _, oa, sa, start, u, calls, backend = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == 'nccl'
    assert calls == {'all_gather_into_tensor': STEPS, 'all_gather_list': 0}, calls
    import hmpc
    d = _inputs(0, PER_RANK, torch.device('cuda', 0), N, True)
    ctx1 = _ctx(hmpc, N)
    out = ctx1.solve_device(d['x_in'], d['x_lin'], d['x_ref'], d['pf'], d['C'], mu=d['mu'])
    torch.cuda.synchronize()
    assert np.array_equal(sa, out['status'].cpu().numpy())
    assert np.array_equal(oa, out['obj'].cpu().numpy())
    assert np.array_equal(u, out['u'].cpu().numpy())
    ctx1.close()
