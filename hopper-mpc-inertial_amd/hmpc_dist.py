"""Multi-GPU layout of the batched solve.

One process per GPU.  The global batch is split into contiguous shards of
``per_rank`` instances; rank r draws instances [r*per_rank, (r+1)*per_rank)
from (seed, global index) (hmpc_plan.sample_instances(start=...)), so a
G-GPU run solves exactly the instances a 1-GPU run would, bit for bit.  The
solve itself has no data-path collective; the one exchange step is an
all-gather of each instance's objective (fp64) and status (int32), over RCCL
(xGMI) on the GPU path and gloo in the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_start(rank: int, per_rank: int) -> int:
    return rank * per_rank


def strong_shard(global_batch: int, world: int, rank: int):
    """(start, count) of rank's contiguous shard of a fixed global batch
    (strong scaling, BASELINE configs[3]: 262144 instances over 2/4/8 GPUs);
    the first global_batch % world ranks take one instance more."""
    base, extra = divmod(global_batch, world)
    count = base + (1 if rank < extra else 0)
    start = rank * base + min(rank, extra)
    return start, count


def allgather_results(obj: torch.Tensor, status: torch.Tensor, out_obj=None, out_status=None):
    """Concatenate every rank's (obj, status) in rank order on every rank."""
    world = dist.get_world_size()
    n = obj.numel()
    if out_obj is None:
        out_obj = torch.empty(n * world, dtype=obj.dtype, device=obj.device)
    if out_status is None:
        out_status = torch.empty(n * world, dtype=status.dtype, device=status.device)
    if dist.get_backend() == 'nccl':
        dist.all_gather_into_tensor(out_obj, obj.contiguous())
        dist.all_gather_into_tensor(out_status, status.contiguous())
    else:
        dist.all_gather(list(out_obj.view(world, n).unbind(0)), obj.contiguous())
        dist.all_gather(list(out_status.view(world, n).unbind(0)), status.contiguous())
    return out_obj, out_status


class ResultExchange:
    """The exchange step of a repeated batched solve, pipelined.

    Each slot is ONE byte buffer per rank, ``[obj (8n B) | status (4n B)]``
    (n = the largest rank's count, padded to 8 B):
    the solve writes its objective and status straight into the slot's views
    (``outputs()``), and ``exchange()`` all-gathers the whole buffer -- one
    collective per step instead of two.  On CUDA/RCCL the all-gather runs on
    a side stream after an event of the solve's stream, so step k's exchange
    overlaps step k+1's solve (which writes the other slot); a slot is
    reused only after its previous all-gather has completed (event wait on
    the solve stream).  ``results(slot)`` returns every rank's (obj, status)
    in rank order.  On gloo (the CPU tests) the exchange is synchronous.
    """

    def __init__(self, n: int, device, nslots: int = 2, counts=None):
        """n: this rank's instance count.  counts: every rank's count (rank
        order) when they differ -- a strong-scaling shard of a global batch
        the world size does not divide (hmpc_dist.strong_shard).  Every
        rank's slot is then sized to the largest count, since the collective
        needs equal sizes; results() trims the padding."""
        self.n, self.world = n, dist.get_world_size()
        self.counts = list(counts) if counts is not None else [n] * self.world
        if len(self.counts) != self.world or self.counts[dist.get_rank()] != n:
            raise ValueError(f'counts {self.counts} do not match rank {dist.get_rank()} with n = {n}')
        self.cap = max(self.counts)
        # bytes per rank: [obj 8 cap | status 4 cap], padded to 8 B so every
        # rank's row of the gathered buffer is float64-aligned
        self.slot = 8 * self.cap + ((4 * self.cap + 7) // 8) * 8
        self.device = torch.device(device)
        self.cuda = self.device.type == 'cuda'
        self.nslots = nslots
        # unused tail of a short rank's slot: zero, so the padding that
        # travels is deterministic
        self.send = [torch.zeros(self.slot, dtype=torch.uint8, device=self.device)
                     for _ in range(nslots)]
        self.recv = [torch.empty(self.world * self.slot, dtype=torch.uint8, device=self.device)
                     for _ in range(nslots)]
        self.stream = torch.cuda.Stream(self.device) if self.cuda else None
        self.done = [None] * nslots
        self.k = 0
        # which collective ran, by path (checked by bench.py and the tests:
        # on the nccl (= RCCL) backend the exchange must be the one
        # all_gather_into_tensor, never the list fallback)
        self.backend = dist.get_backend()
        self.calls = {'all_gather_into_tensor': 0, 'all_gather_list': 0}

    def outputs(self):
        """(obj float64 [n], status int32 [n]) views of the next slot's send
        buffer; the solve stream first waits for that slot's last exchange."""
        s = self.k % self.nslots
        if self.cuda and self.done[s] is not None:
            torch.cuda.current_stream(self.device).wait_event(self.done[s])
        buf = self.send[s]
        c8 = 8 * self.cap
        return buf[:8 * self.n].view(torch.float64), buf[c8:c8 + 4 * self.n].view(torch.int32)

    def exchange(self) -> int:
        """All-gather the slot the last ``outputs()`` handed out; returns it."""
        s = self.k % self.nslots
        self.k += 1
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ev)
                self._gather(s)
                done = torch.cuda.Event()
                done.record(self.stream)
            self.done[s] = done
        else:
            self._gather(s)
        return s

    def _gather(self, s):
        if self.backend == 'nccl':
            dist.all_gather_into_tensor(self.recv[s], self.send[s])
            self.calls['all_gather_into_tensor'] += 1
        else:
            self.calls['all_gather_list'] += 1
            dist.all_gather(list(self.recv[s].view(self.world, self.slot).unbind(0)),
                            self.send[s])

    def wait(self):
        """Make the current stream wait for every outstanding exchange."""
        if self.cuda:
            cur = torch.cuda.current_stream(self.device)
            for d in self.done:
                if d is not None:
                    cur.wait_event(d)

    def results(self, slot: int):
        """(obj [sum counts] float64, status [sum counts] int32) of a slot, in
        rank order (each rank's padding trimmed)."""
        r = self.recv[slot].view(self.world, self.slot)
        c8 = 8 * self.cap
        obj = torch.cat([r[i, :8 * c].contiguous().view(torch.float64) for i, c in enumerate(self.counts)])
        st = torch.cat([r[i, c8:c8 + 4 * c].contiguous().view(torch.int32) for i, c in enumerate(self.counts)])
        return obj, st
