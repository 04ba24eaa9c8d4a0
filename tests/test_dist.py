"""Multi-process path on CPU with gloo, world_size 2 and 4: each rank
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
    # ... exchanged with uneven per-rank counts (world does not divide the
    # global batch): slots sized to the largest shard, padding trimmed
    counts = [hmpc_dist.strong_shard(2 * PER_RANK + 1, world, r)[1] for r in range(world)]
    assert len(set(counts)) == 2
    ux = hmpc_dist.ResultExchange(gcount, 'cpu', counts=counts)
    o, s = ux.outputs()
    o.copy_(torch.from_numpy(sobj))
    s.copy_(torch.from_numpy(sst))
    uobj, ust = ux.results(ux.exchange())
    q.put((rank, oa.numpy().copy(), sa.numpy().copy(), po.numpy().copy() / 3, ps.numpy().copy() - 2,
           gstart, gcount, sobj, sst, uobj.numpy().copy(), ust.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4])
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
    assert shards[0][0] == 0
    for lo, hi in zip(shards, shards[1:]):
        assert lo[0] + lo[1] == hi[0]
    assert shards[-1][0] + shards[-1][1] == 2 * PER_RANK + 1
    assert np.array_equal(np.concatenate([sh[2] for sh in shards]), gobj)
    assert np.array_equal(np.concatenate([sh[3] for sh in shards]), gst)
    for r in res:   # the uneven exchange: every rank holds the whole global batch
        assert np.array_equal(r[9], gobj)
        assert np.array_equal(r[10], gst)


class _FakeNccl:
    """Stands in for torch.distributed on the nccl (RCCL) backend, rank 0 of
    a world of 3 with uneven counts: all_gather_into_tensor fills every
    rank's slot, the other ranks' with a payload built from their rank."""

    def __init__(self, counts, rank=0):
        self.counts, self.rank, self.seen = counts, rank, []

    def get_world_size(self):
        return len(self.counts)

    def get_rank(self):
        return self.rank

    def get_backend(self):
        return 'nccl'

    @staticmethod
    def payload(r, n, cap):
        buf = torch.zeros(8 * cap + ((4 * cap + 7) // 8) * 8, dtype=torch.uint8)
        buf[:8 * n].view(torch.float64).copy_(torch.arange(n, dtype=torch.float64) + 1000.0 * r)
        buf[8 * cap:8 * cap + 4 * n].view(torch.int32).copy_(torch.full((n,), r, dtype=torch.int32))
        return buf

    def all_gather_into_tensor(self, out, inp):
        cap = max(self.counts)
        slot = 8 * cap + ((4 * cap + 7) // 8) * 8
        self.seen.append((out.numel(), inp.numel(), out.dtype, inp.dtype, out.is_contiguous()))
        assert out.numel() == len(self.counts) * inp.numel() == len(self.counts) * slot
        v = out.view(len(self.counts), slot)
        for r, n in enumerate(self.counts):
            v[r].copy_(inp if r == self.rank else self.payload(r, n, cap))

    def all_gather(self, *a, **k):
        raise AssertionError('the nccl path must not take the list all-gather')


def test_nccl_exchange_buffer_views(monkeypatch):
    """The RCCL branch of ResultExchange._gather (never executed on this
    CPU-only box) builds the right buffers: one all_gather_into_tensor per
    step of world x 12 cap bytes, obj / status views at the right offsets,
    results() trimming each rank's padding."""
    import hmpc_dist
    counts = [5, 4, 4]
    fake = _FakeNccl(counts)
    monkeypatch.setattr(hmpc_dist, 'dist', fake)
    ex = hmpc_dist.ResultExchange(counts[0], 'cpu', counts=counts)
    assert ex.backend == 'nccl' and ex.cap == 5
    for step in range(3):
        o, s = ex.outputs()
        assert o.numel() == 5 and s.numel() == 5 and o.dtype == torch.float64 and s.dtype == torch.int32
        o.copy_(torch.arange(5, dtype=torch.float64) + 0.5 * step)
        s.copy_(torch.full((5,), 7, dtype=torch.int32))
        slot = ex.exchange()
    assert ex.calls == {'all_gather_into_tensor': 3, 'all_gather_list': 0}
    assert all(sz == (3 * 64, 64, torch.uint8, torch.uint8, True) for sz in fake.seen)
    obj, st = ex.results(slot)
    assert obj.numel() == st.numel() == sum(counts)
    np.testing.assert_array_equal(obj[:5].numpy(), np.arange(5) + 1.0)
    np.testing.assert_array_equal(obj[5:9].numpy(), np.arange(4) + 1000.0)
    np.testing.assert_array_equal(obj[9:].numpy(), np.arange(4) + 2000.0)
    np.testing.assert_array_equal(st.numpy(), [7] * 5 + [1] * 4 + [2] * 4)
    with pytest.raises(ValueError):
        hmpc_dist.ResultExchange(4, 'cpu', counts=counts)   # rank 0 holds 5
