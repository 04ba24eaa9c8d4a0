"""Multi-process path on CPU with gloo, world_size 2: each rank
draws its contiguous shard from (seed, global index), solves it (here with the
oracle's C port standing in for the GPU kernel) and all-gathers objective +
status; every rank must end with exactly the single-process result."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PER_RANK = 96
N = 10


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _solve(start, count):
    import hmpc_plan
    from oracle import port
    inst = hmpc_plan.sample_instances(count, N, curve=True, seed=31, mu_sweep=(0.3, 1.2),
                                      start=start)
    r = port.solve_batch('3f', N, *[inst[k] for k in ('x_in', 'x_lin', 'x_ref', 'pf', 'C')],
                         mu=inst['mu'])
    return r['obj'], r['status']


def _worker(rank, world, port, q):
    import sys
    for p in (os.path.join(ROOT, 'hopper-mpc-inertial_amd'), ROOT):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import hmpc_dist
    obj, st = _solve(hmpc_dist.shard_start(rank, PER_RANK), PER_RANK)
    oa, sa = hmpc_dist.allgather_results(torch.from_numpy(obj), torch.from_numpy(st))
    # the bench's pipelined exchange: packed [obj | status] slots, two steps
    ex = hmpc_dist.ResultExchange(PER_RANK, 'cpu')
    slots = []
    for step in range(3):
        o, s = ex.outputs()
        o.copy_(torch.from_numpy(obj) * (step + 1))
        s.copy_(torch.from_numpy(st) + step)
        slots.append(ex.exchange())
    ex.wait()
    po, ps = ex.results(slots[2])   # slot 0 again: step 2 overwrote step 0
    # gloo takes the list all-gather; the nccl (RCCL) path is counted apart
    assert ex.backend == 'gloo'
    assert ex.calls == {'all_gather_into_tensor': 0, 'all_gather_list': 3}, ex.calls
    # strong scaling: a fixed global batch in contiguous shards
    gstart, gcount = hmpc_dist.strong_shard(2 * PER_RANK + 1, world, rank)
    sobj, sst = _solve(gstart, gcount)
    q.put((rank, oa.numpy().copy(), sa.numpy().copy(), po.numpy().copy() / 3, ps.numpy().copy() - 2,
           gstart, gcount, sobj, sst))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2])
def test_sharded_allgather_equals_single_process(world):
    import subprocess
    subprocess.check_call(['make', '-s', '-C', os.path.join(ROOT, 'oracle')])
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    obj_ref, st_ref = _solve(0, PER_RANK * world)
    for _, oa, sa, po, ps, *_ in res:
        assert np.array_equal(oa, obj_ref)
        assert np.array_equal(sa, st_ref)
        assert np.allclose(po, obj_ref, rtol=1e-15, atol=0)
        assert np.array_equal(ps, st_ref)
    # the strong-scaling shards tile [0, 2 PER_RANK + 1) and reproduce the
    # single-process solve bit for bit
    gobj, gst = _solve(0, 2 * PER_RANK + 1)
    shards = sorted((r[5], r[6], r[7], r[8]) for r in res)
    assert shards[0][0] == 0 and shards[0][0] + shards[0][1] == shards[1][0]
    assert shards[1][0] + shards[1][1] == 2 * PER_RANK + 1
    assert np.array_equal(np.concatenate([sh[2] for sh in shards]), gobj)
    assert np.array_equal(np.concatenate([sh[3] for sh in shards]), gst)
