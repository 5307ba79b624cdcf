"""Multi-GPU helpers (one process per GPU, torch.distributed over RCCL/xGMI; gloo on CPU tests).

SURVEY.md §8e: the hot path shards naturally —
* RTN / fake-quant / pack and DSv3 expert linears: independent units -> ``lpt_shard``;
* AWQ with ``quant_out: False``: blocks independent given the float activations ->
  ``block_shard`` (each rank transforms its own blocks, then ``broadcast_block`` publishes the
  quantized weights from the owner: the only collective is the gather of quantized shards);
* GPTQ within a block: rows independent given U -> ``row_shard`` + ``gather_rows``.
The reference's own data-parallel semantics (replicas with averaged statistics) are kept by
``allreduce_mean_`` and ``awq_pick_best`` (awq.py:255-273) for drop-in DP runs.
"""
from __future__ import annotations

import heapq

import torch
import torch.distributed as dist


def dist_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def block_shard(n_blocks: int, rank: int, world: int) -> list[int]:
    """Round-robin block ownership (rank r owns r, r+world, ...)."""
    return list(range(rank, n_blocks, world))


def lpt_shard(costs: list[float], world: int) -> list[list[int]]:
    """Longest-processing-time assignment of independent units to ranks (deterministic)."""
    heap = [(0.0, r) for r in range(world)]
    out = [[] for _ in range(world)]
    for i in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + costs[i], r))
    return [sorted(o) for o in out]


def row_shard(rows: int, rank: int, world: int, align: int = 1) -> tuple[int, int]:
    """Contiguous [start, end) row range of this rank (balanced), in units of ``align`` rows
    (a per-tensor FP8 clip scale spans one 256- or 64-row batch, auto_clip.py:108)."""
    units = -(-rows // align)
    base, rem = divmod(units, world)
    start = rank * base + min(rank, rem)
    end = start + base + (1 if rank < rem else 0)
    return min(start * align, rows), min(end * align, rows)


def allreduce_mean_(t: torch.Tensor) -> torch.Tensor:
    """all_reduce(SUM) then / world_size, in place (gptq.py:292-295, auto_clip.py:72-76)."""
    rank, world = dist_world()
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t /= world
    return t


def awq_pick_best(best_error: float, best_scales: torch.Tensor) -> torch.Tensor:
    """awq.py:255-273: global min loss, highest rank within 1e-5 of it wins, its scales are
    broadcast to every rank."""
    rank, world = dist_world()
    if world == 1:
        return best_scales
    dev = best_scales.device
    err = torch.tensor([best_error], dtype=torch.float64, device=dev)
    dist.all_reduce(err, op=dist.ReduceOp.MIN)
    gbest = err.item()
    who = torch.tensor([rank if abs(best_error - gbest) < 1e-5 else -1], device=dev)
    dist.all_reduce(who, op=dist.ReduceOp.MAX)
    src = int(who.item())
    out = best_scales.clone() if rank == src else torch.zeros_like(best_scales)
    dist.broadcast(out, src=src)
    return out


def gather_rows(local: torch.Tensor, rows: int, align: int = 1) -> torch.Tensor:
    """Reassemble a row-sharded matrix (row_shard layout) on every rank."""
    rank, world = dist_world()
    if world == 1:
        return local
    sizes = [row_shard(rows, r, world, align) for r in range(world)]
    maxr = max(e - s for s, e in sizes)
    pad = torch.zeros((maxr,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return torch.cat([p[: e - s] for p, (s, e) in zip(parts, sizes)], dim=0)


def broadcast_block(block: torch.nn.Module, owner: int):
    """Publish an owner-transformed block's parameters and buffers to every rank."""
    rank, world = dist_world()
    if world == 1:
        return
    for t in block.parameters():
        dist.broadcast(t.data, src=owner)
    # buffers the owner's transform registered (e.g. static act qparams buf_act_*) may not
    # exist on the other ranks: publish the owner's buffer list first, create what is missing
    spec = [None]
    if rank == owner:
        spec = [[(mn, bn, tuple(b.shape), str(b.dtype).split('.')[-1])
                 for mn, m in block.named_modules() for bn, b in m.named_buffers(recurse=False)
                 if b is not None]]
    dist.broadcast_object_list(spec, src=owner)
    mods = dict(block.named_modules())
    dev = next(block.parameters(), next(block.buffers(), None))
    dev = dev.device if dev is not None else torch.device('cpu')
    for mn, bn, shape, dt in spec[0]:
        m = mods[mn]
        b = m._buffers.get(bn)
        if b is None or tuple(b.shape) != shape or str(b.dtype).split('.')[-1] != dt:
            m.register_buffer(bn, torch.empty(shape, dtype=getattr(torch, dt), device=dev))
        dist.broadcast(m._buffers[bn].data, src=owner)


def ring_groups(world: int):
    """One process group per ring edge (r, r + 1 mod world), created on every rank in the same
    order (group creation is collective): the block hand-off of the pipelined shard_blocks
    loop uses edge r to pass block activations from rank r to rank r + 1."""
    return [dist.new_group([r, (r + 1) % world]) for r in range(world)]


def pass_tensors(tensors, src: int, group):
    """Hand a list of device tensors from `src` to the other rank of a ring-edge group (a
    broadcast within the pair: P2P over xGMI under RCCL, and valid on gloo as well). On the
    receiving rank `tensors` are buffers of the right shapes and dtypes, filled in place."""
    for t in tensors:
        dist.broadcast(t, src=src, group=group)

