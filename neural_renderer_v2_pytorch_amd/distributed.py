"""Batch sharding across the GPUs of a node.

The rasterizer has no cross-item dependency (every kernel indexes its item by blockIdx.y), so a
batch shards by items: rank r of G renders items [shard_range(B, r, G)) on its own GPU with no
communication on the data path.  Two collectives exist only where the path has a real exchange:

* gather_images -- the rendered shards are assembled on every rank with one
  all_gather_into_tensor (RCCL over xGMI on MI355X; one message of B/G * C * s * s floats per rank);
* allreduce_shared_grads -- parameters shared by all items (one mesh rendered from several views,
  one texture atlas) get their gradient summed across ranks with all_reduce(SUM).

One process per GPU, launched by torchrun; the backend is "nccl" (= RCCL on ROCm) on GPUs and
"gloo" in the CPU tests.
"""
import torch
import torch.distributed as dist


def world(group=None):
    """(rank, world size) within `group` (the default group when None); (0, 1) without a
    process group.  A rank outside `group` gets a ValueError: torch reports it as rank -1, which
    the shard arithmetic would otherwise silently use."""
    if dist.is_available() and dist.is_initialized():
        rank = dist.get_rank(group)
        if rank < 0:
            raise ValueError("this process (global rank %d) is not a member of the given group" % dist.get_rank())
        return rank, dist.get_world_size(group)
    return 0, 1


def shard_range(batch_size, rank, world_size):
    """Contiguous item range [start, end) of `rank`; sizes differ by at most one item."""
    base, extra = divmod(batch_size, world_size)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard(tensor, rank=None, world_size=None, dim=0):
    """This rank's slice of a batch-major tensor (a view, no copy)."""
    if rank is None or world_size is None:
        rank, world_size = world()
    start, end = shard_range(tensor.shape[dim], rank, world_size)
    return tensor.narrow(dim, start, end - start)


def gather_images(local, batch_size=None, group=None):
    """All-gather batch shards [b_r, ...] into the full batch [B, ...] on every rank.

    Uneven shards (B not divisible by the group size) are padded to the largest shard for the
    collective and trimmed afterwards.  Shards are ordered by rank within `group`."""
    rank, ws = world(group)
    if ws == 1:
        return local
    if batch_size is None:
        sizes = torch.tensor([local.shape[0]], device=local.device, dtype=torch.int64)
        allsizes = [torch.zeros_like(sizes) for _ in range(ws)]
        dist.all_gather(allsizes, sizes, group=group)
        batch_size = int(sum(int(x) for x in allsizes))
    ranges = [shard_range(batch_size, r, ws) for r in range(ws)]
    cap = max(e - s for s, e in ranges)
    src = local.contiguous()
    if src.shape[0] != cap:
        pad = torch.zeros((cap - src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        src = torch.cat([src, pad], 0)
    out = torch.empty((ws * cap,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    if all(e - s == cap for s, e in ranges):
        return out
    return torch.cat([out[r * cap:r * cap + (e - s)] for r, (s, e) in enumerate(ranges)], 0)


def allreduce_shared_grads(params, group=None):
    """Sum the gradients of parameters shared by every rank's items (in place).

    Every rank issues the same collectives in the same order: a parameter that requires grad but
    whose .grad is None on this rank (an empty shard, or a branch this rank did not take)
    contributes zeros, and its .grad is materialised, so no rank skips an all_reduce the others
    enter.  Parameters that do not require grad (frozen) are skipped on every rank alike and keep
    .grad None, so optimisers (weight decay, momentum) leave them alone."""
    _, ws = world(group)
    if ws == 1:
        return
    for p in params:
        if p is None or not p.requires_grad:
            continue
        if p.grad is None:
            p.grad = torch.zeros_like(p)
        dist.all_reduce(p.grad, op=dist.ReduceOp.SUM, group=group)
