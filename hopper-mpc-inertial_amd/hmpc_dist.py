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
