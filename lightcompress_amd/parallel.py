"""Multi-GPU helpers (one process per GPU, torch.distributed over RCCL/xGMI; gloo on CPU tests).

SURVEY.md §8e: the hot path shards naturally —
* RTN / fake-quant / pack and DSv3 expert linears: independent units -> ``lpt_shard``;
* AWQ with ``quant_out: False``: blocks independent given the float activations ->
  ``block_shard`` (each rank transforms its own blocks, then ``broadcast_block`` publishes the
  quantized weights from the owner: the only collective is the gather of quantized shards);
* GPTQ within a block: rows independent given U -> ``row_shard`` + ``gather_rows``.
The reference's own data-parallel semantics (replicas with averaged statistics) are kept by
``allreduce_mean_`` and ``awq_pick_best`` (awq.py:255-273) for drop-in DP runs.

Independent-unit deploys (data-free RTN, DSv3 experts) run as ``shard_units``: every rank
real-quants the units ``residency.Ownership`` assigns it (LPT on parameter counts) and the
packed results are published with ``publish`` -- one flat byte broadcast per (block, owner),
never a float weight.
"""
from __future__ import annotations

import heapq
import importlib

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
    _, world = dist_world()
    if world == 1:
        return local
    return gather_ranges(local, [row_shard(rows, r, world, align) for r in range(world)])


def gather_ranges(local: torch.Tensor, sizes) -> torch.Tensor:
    """Reassemble rows held as contiguous [start, end) ranges, rank r holding sizes[r], on
    every rank (one all_gather of equal padded parts, concatenated in rank order)."""
    rank, world = dist_world()
    if world == 1:
        return local
    if local.shape[0] != sizes[rank][1] - sizes[rank][0]:
        raise ValueError(f'rank {rank} holds {local.shape[0]} rows, its range is {sizes[rank]}')
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



def planned_mode(config, world: int) -> str:
    """The parallel mode a run of `config` takes at `world` ranks, known before the model is
    built (BlockwiseOpt.parallel_mode decides the same from the algorithm object): the
    YAML's special.parallel, else shard_units for a data-free run (no calib section,
    llmc/__main__.py:42), shard_blocks when quant_out is off, else the algorithm's own
    sequential mode."""
    if world == 1:
        return 'single'
    q = config['quant']
    mode = (q.get('special', {}) or {}).get('parallel', None)
    if mode:
        return mode
    if not config.get('calib', False):
        return 'shard_units'
    if not q.get('quant_out', False):
        return 'shard_blocks'
    from .registry import ALGO_REGISTRY
    return getattr(ALGO_REGISTRY[q['method']], 'sequential_parallel_mode', 'replicate')


_PLAIN = (int, float, str, bool, tuple, torch.Size, torch.dtype, type(None))


def _plain_attrs(m):
    return {k: v for k, v in m.__dict__.items()
            if not k.startswith('_') and k != 'training' and isinstance(v, _PLAIN)}


def _opaque_attrs(m):
    """Names of a module's attributes that cannot travel as a spec (callables such as a fake-quant
    module's a_qdq, dicts such as its debug_print): the non-owner rebuilds them locally."""
    return sorted(k for k, v in m.__dict__.items()
                  if not k.startswith('_') and k != 'training' and not isinstance(v, _PLAIN))


def _slots(m, recurse):
    mods = m.named_modules() if recurse else [('', m)]
    for mn, mod in mods:
        for kind in ('_parameters', '_buffers'):
            for tn, t in getattr(mod, kind).items():
                yield mn, mod, kind, tn, t


def _dt(t):
    return str(t.dtype).split('.')[-1]


@torch.no_grad()
def publish(block: torch.nn.Module, assign: dict, rest_owner: int | None = None,
            local_attrs: dict | None = None):
    """After each rank replaced the block's modules it owns (``assign``: module name relative
    to the block -> owner rank), give every rank the same block: the non-owners rebuild each
    module as an empty instance of the owner's class (same plain attributes, parameters and
    buffers of the owner's shapes and dtypes; their old modules are dropped unread), then
    every owner broadcasts ALL its modules' tensors as one flat byte buffer. With
    ``rest_owner`` the block's other tensors (norms, ...) come from that rank the same way,
    buffers it registered included. Attributes that are not plain values (a fake-quant
    module's ``a_qdq`` callable, its ``debug_print`` dict) cannot be shipped: a rebuilt module
    takes them from ``local_attrs`` (the local algorithm's replacement params -- the same
    callables the owner used), and a missing one raises here rather than at the first forward.
    Collectives: one all_gather_object of the specs, one broadcast per owner with data."""
    rank, world = dist_world()
    if world == 1:
        return
    mine = []
    for n, r in sorted(assign.items()):
        if r != rank:
            continue
        m = block.get_submodule(n)
        mine.append((n, type(m).__module__, type(m).__qualname__, _plain_attrs(m),
                     [(kind, tn, None if t is None else tuple(t.shape),
                       None if t is None else _dt(t))
                      for _, _, kind, tn, t in _slots(m, recurse=False)], _opaque_attrs(m)))
    rest = None
    if rest_owner == rank:
        under = tuple(f'{n}.' for n in assign)
        rest = [(mn, kind, tn, tuple(t.shape), _dt(t))
                for mn, _, kind, tn, t in _slots(block, recurse=True)
                if t is not None and mn not in assign and not mn.startswith(under)]
    specs = [None] * world
    dist.all_gather_object(specs, (mine, rest))
    dev = next((t.device for _, _, _, _, t in _slots(block, True)
                if t is not None and not t.is_meta), torch.device('cpu'))
    for r, (mods, rst) in enumerate(specs):
        if r == rank:
            continue
        for n, modname, qual, attrs, tensors, opaque in mods:
            cls = importlib.import_module(modname)
            for part in qual.split('.'):
                cls = getattr(cls, part)
            m = cls.__new__(cls)
            torch.nn.Module.__init__(m)
            for kind, tn, shape, dt in tensors:
                t = None if shape is None else torch.empty(shape, dtype=getattr(torch, dt),
                                                           device=dev)
                if kind == '_parameters':
                    m.register_parameter(tn, None if t is None else
                                         torch.nn.Parameter(t, requires_grad=False))
                else:
                    m.register_buffer(tn, t)
            for k, v in attrs.items():
                setattr(m, k, v)
            for k in opaque:
                if local_attrs is None or k not in local_attrs:
                    raise RuntimeError(f'publish: attribute {k!r} of {qual} {n!r} (owner rank '
                                       f'{r}) is not a plain value and no local value was '
                                       'given (local_attrs)')
                setattr(m, k, local_attrs[k])
            parent_name, _, child = n.rpartition('.')
            parent = block.get_submodule(parent_name) if parent_name else block
            old = parent._modules.get(child)
            setattr(parent, child, m)
            if old is not None:
                from .base_model import retire_module
                retire_module(old)
        for mn, kind, tn, shape, dt in (rst or []):
            mod = block.get_submodule(mn) if mn else block
            t = getattr(mod, kind).get(tn)
            if t is None or tuple(t.shape) != shape or _dt(t) != dt or t.is_meta:
                new = torch.empty(shape, dtype=getattr(torch, dt), device=dev)
                if kind == '_parameters' and t is not None:
                    t.data = new
                elif kind == '_parameters':
                    mod.register_parameter(tn, torch.nn.Parameter(new, requires_grad=False))
                else:
                    mod.register_buffer(tn, new)
    for r, (mods, rst) in enumerate(specs):
        ts = []
        for n, _, _, _, tensors, _ in mods:
            m = block.get_submodule(n)
            ts += [getattr(m, kind)[tn] for kind, tn, shape, _ in tensors if shape is not None]
        for mn, kind, tn, _, _ in (rst or []):
            ts.append(getattr(block.get_submodule(mn) if mn else block, kind)[tn])
        sizes = [t.numel() * t.element_size() for t in ts]
        total = sum(sizes)
        if total == 0:
            continue
        if r == rank:
            flat = torch.cat([t.detach().contiguous().reshape(-1).view(torch.uint8)
                              for t in ts])
        else:
            flat = torch.empty(total, dtype=torch.uint8, device=dev)
        dist.broadcast(flat, src=r)
        if r != rank:
            off = 0
            for t, nb in zip(ts, sizes):
                dst = t.data if t.data.is_contiguous() else torch.empty_like(
                    t.data, memory_format=torch.contiguous_format)
                dst.reshape(-1).view(torch.uint8).copy_(flat[off:off + nb])
                if dst is not t.data:
                    t.data.copy_(dst)
                off += nb
