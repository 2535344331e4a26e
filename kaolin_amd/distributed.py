"""View sharding across GPUs (one process per GPU) and the one exchange step of the path.

The reference has no distributed code.  DIB-R views are independent through the
whole forward and the per-view backward kernels (no cross-view terms: rasterization_cuda.cu:62,
dibr_soft_mask_cuda.cu:47-51), so views are sharded in contiguous blocks and the only exchange is
the sum over views of the shared mesh parameters' gradients -- the ``.repeat(batch_size, 1, 1)``
backward of the reference training loop (examples/tutorial/ian_dibr.py:225-229) -- done as ONE
bucketed all-reduce (RCCL over xGMI with backend "nccl"; gloo on CPU for tests).
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise torch.distributed from RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* when
    WORLD_SIZE > 1.  Returns (rank, world_size, local_rank)."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', str(rank)))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = 'nccl' if torch.cuda.is_available() else 'gloo'
        kw = {}
        if backend == 'nccl':
            torch.cuda.set_device(local)
            kw['device_id'] = torch.device('cuda', local)
        dist.init_process_group(backend=backend, init_method='env://', rank=rank,
                                world_size=world, **kw)
    return rank, world, local


def shard_views(total_views, rank, world):
    """Contiguous block of views for `rank`: (first_view, num_views).  Remainders go to the
    lowest ranks, so every view is rendered exactly once."""
    base, rem = divmod(total_views, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def allreduce_grads_(tensors, group=None):
    """Sum `tensors` (e.g. shared-parameter .grad) over all ranks in place, as one flat bucket
    (one collective per step).  No-op when not distributed."""
    tensors = [t for t in tensors if t is not None]
    if not tensors or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return tensors
    if len(tensors) == 1 and tensors[0].is_contiguous():  # in place: no pack / unpack kernels
        dist.all_reduce(tensors[0], op=dist.ReduceOp.SUM, group=group)
        return tensors
    flat = torch.cat([t.reshape(-1) for t in tensors])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    off = 0
    for t in tensors:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t))
        off += n
    return tensors
