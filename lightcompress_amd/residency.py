"""Where the decoder blocks live: HBM-resident, streamed from pinned host memory, or owned by
one rank of a sharded run (the other ranks never allocate them).

The reference keeps the whole model on the host and moves one block at a time: ``block.cuda()``
at the start of ``block_opt`` and ``block.cpu()`` at its end (base_blockwise_quantization.py:
397, 418), the same around every block of ``deploy`` (``replace_module_all`` with
``keep_device=False``, models/base_model.py:380-390). That is how it quantizes DeepSeek-V3/R1
671B "on a single GPU" (README.md:43), with every copy synchronous on the compute stream.

MI355X-first placements (YAML ``model.residency`` / ``model.materialize``):

* ``device``: every block resident in HBM (288 GB holds Llama-3-70B bf16) -- no copies at all;
  the default whenever the model fits.
* ``stream``: block tensors host-resident in pinned memory; ``BlockStreamer`` uploads block
  i + 1 on an H2D side stream while block i is transformed on the compute stream, and writes
  block i back on a D2H side stream afterwards (at most three blocks in HBM: the one being
  transformed, the next one arriving, the previous one leaving). Same kernels on the same
  operands, so results are bit-identical to ``device``.
* ``owned`` (world > 1, sharded plans): each rank materialises only the blocks / units it owns
  (``Ownership``); everything else stays on the meta device -- for a 671B FP8 model over 8
  ranks, ~84 GB per rank instead of 671 GB on every rank.
"""
from __future__ import annotations

import re
import sys
import time
import weakref

import torch
import torch.nn as nn

_EXPERT = re.compile(r'^(.*\bexperts\.\d+)\.')


def unit_key(linear_name: str) -> str:
    """The independent unit a block linear belongs to: a routed expert's
    linears form one unit (EP-style: an expert's gate / up / down stay on one rank), every
    other linear is its own unit."""
    m = _EXPERT.match(linear_name)
    return m.group(1) if m else linear_name


def _tensor_slots(module: nn.Module):
    """(owner module, '_parameters' | '_buffers', name, tensor) of every tensor under module."""
    for m in module.modules():
        for kind in ('_parameters', '_buffers'):
            for n, t in getattr(m, kind).items():
                if t is not None:
                    yield m, kind, n, t


def _install(m: nn.Module, kind: str, n: str, t: torch.Tensor):
    if kind == '_parameters':
        p = m._parameters[n]
        if p.is_meta or t.is_meta:      # meta <-> real (loading, dropping): a new Parameter
            m._parameters[n] = nn.Parameter(t, requires_grad=p.requires_grad)
        else:
            p.data = t      # keeps the Parameter object (hooks, subsets hold it)
    else:
        m._buffers[n] = t


def _scrub(block: nn.Module):
    """Drop device-side memos hung on modules as plain attributes (the fused forwards' stage
    outputs, expert row maps, precomputed column groups): they would pin HBM after eviction and
    are rebuilt on demand."""
    for m in block.modules():
        for k in [k for k in m.__dict__ if k.startswith('_lcq_')]:
            v = m.__dict__[k]
            if torch.is_tensor(v) or isinstance(v, (tuple, list, dict)):
                del m.__dict__[k]


class BlockStreamer:
    """Pinned-host <-> HBM streaming of decoder blocks with copy/compute overlap.

    ``fetch(i)`` makes block i device-resident on the compute stream (waiting for its prefetch,
    or uploading it now); ``prefetch(i)`` starts block i's upload on the H2D stream;
    ``evict(i)`` enqueues block i's write-back on the D2H stream (after everything the compute
    stream has issued so far) and points its modules at the host copies; ``drain()`` waits for
    every write-back (call it before the host reads the tensors). Module and Parameter objects
    never change, only their ``.data`` -- hooks, subset dicts and the algorithms' references
    stay valid."""

    def __init__(self, blocks, device):
        self.blocks = blocks
        self.dev = torch.device(device)
        self.h2d = torch.cuda.Stream(device=self.dev)
        self.d2h = torch.cuda.Stream(device=self.dev)
        self.pending = {}        # block -> (event, moves)
        self.resident = set()
        self.host = {}           # (id(module), kind, name) -> (weakref(module), pinned host)
        self.stats = {'h2d_bytes': 0, 'd2h_bytes': 0, 'fetches': 0, 'prefetched': 0,
                      'pin_alloc_bytes': 0, 'pin_alloc_s': 0.0, 'evict_host_s': 0.0,
                      'pin_ahead_bytes': 0, 'pin_recycled_bytes': 0, 'host_new': 0,
                      'host_retyped': 0, 'host_released': 0, 'host_deployed_modules': 0}
        # Fresh page-locked memory costs ~11 ms of host time per 224 MiB (hipHostMalloc at
        # ~20 GiB/s, profiles/r6_stream_gptq.md), and a GPTQ block turns its 7 bf16 linears
        # into FakeQuantLinear with fp32 weights (gptq.py:193) -- 0.87 GB of new host copies
        # per Llama-3-8B block, then the deploy's new modules as much again. Remedies, none
        # changing a byte: replaced modules' host tensors are handed to their replacements
        # (evict's pool); copies that still had to be allocated are allocated ahead for the
        # next block on a worker thread (torch.empty releases the GIL) while the GPU works.
        # (A fake-quant deploy of a streamed block builds its modules on the host from the
        # FakeQuantLinear memos: BaseBlockwiseQuantization._deploy_from_memos.)
        self._ahead = []         # futures of [(shape, dtype, pinned tensor)] for the next block
        self._pool = None

    def _take_pinned(self, shape, dtype):
        """A pinned host tensor of (shape, dtype): one allocated ahead if any, else a new one."""
        key = (tuple(shape), dtype)
        for fut in self._ahead:
            bufs = fut.result()   # waits for the worker if it is still allocating
            for j, (shp, dt, t) in enumerate(bufs):
                if (shp, dt) == key:
                    del bufs[j]
                    return t
        t_al = time.perf_counter()
        h = torch.empty(shape, dtype=dtype, pin_memory=True)
        self.stats['pin_alloc_s'] += time.perf_counter() - t_al
        self.stats['pin_alloc_bytes'] += h.numel() * h.element_size()
        return h

    def _allocate_ahead(self, wants):
        """Allocate pinned host tensors for [(shape, dtype)] on the worker thread."""
        if self._pool is None:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix='lcq-pin')
        self._ahead = [f for f in self._ahead if not f.done() or f.result()]
        self.stats['pin_ahead_bytes'] += sum(
            torch.Size(s).numel() * torch.empty((), dtype=d).element_size() for s, d in wants)
        self._ahead.append(self._pool.submit(
            lambda: [(s, d, torch.empty(s, dtype=d, pin_memory=True)) for s, d in wants]))

    def release_ahead(self):
        """Drop host tensors allocated ahead and not used (end of a pass over the blocks)."""
        for fut in self._ahead:
            fut.result()
        self._ahead = []

    def __len__(self):
        return len(self.blocks)

    def pin_all(self):
        """Every block tensor into pinned host memory (async copies need page-locked sources;
        one pass at model load)."""
        for block in self.blocks:
            for m, kind, n, t in _tensor_slots(block):
                if t.is_meta:
                    continue
                if t.device.type != 'cpu':
                    t = t.cpu()
                if not t.is_pinned():
                    t = t.pin_memory()
                _install(m, kind, n, t)
                self.host[(id(m), kind, n)] = (weakref.ref(m), t)

    def _host_of(self, m, kind, n):
        ent = self.host.get((id(m), kind, n))
        return ent[1] if ent is not None and ent[0]() is m else None

    def prefetch(self, i: int):
        if i < 0 or i >= len(self.blocks) or i in self.resident or i in self.pending:
            return
        # after any write-back still in flight (a re-fetch at deploy reads what the D2H stream
        # wrote); nothing on the compute stream produces host data, so the upload does not
        # queue behind it (its allocations come from the H2D stream's own pool)
        self.h2d.wait_stream(self.d2h)
        moves = []
        with torch.cuda.stream(self.h2d):
            for m, kind, n, t in _tensor_slots(self.blocks[i]):
                if t.is_meta or t.device.type == 'cuda':
                    continue
                d = torch.empty(t.shape, dtype=t.dtype, device=self.dev)
                d.copy_(t, non_blocking=True)
                self.stats['h2d_bytes'] += t.numel() * t.element_size()
                moves.append((m, kind, n, d))
        ev = torch.cuda.Event()
        ev.record(self.h2d)
        self.pending[i] = (ev, moves)

    def fetch(self, i: int):
        if i in self.resident:
            return self.blocks[i]
        if i in self.pending:
            self.stats['prefetched'] += 1
        else:
            self.prefetch(i)
        ev, moves = self.pending.pop(i)
        main = torch.cuda.current_stream(self.dev)
        main.wait_event(ev)
        for m, kind, n, d in moves:
            d.record_stream(main)   # allocated on the H2D stream, used on the compute stream
            _install(m, kind, n, d)
        self.resident.add(i)
        self.stats['fetches'] += 1
        return self.blocks[i]

    def evict(self, i: int, dirty: bool = True):
        """Block i back to the host. ``dirty`` False (a forward-only visit): the host copies
        are still current, nothing is copied."""
        if i not in self.resident:
            return
        t_ev = time.perf_counter()
        block = self.blocks[i]
        _scrub(block)
        # host copies of modules replaced since (deploy swaps the linears): their exclusively
        # held tensors serve the new modules' copies of the same shape and dtype (the D2H
        # stream writes them only after the compute stream, which waited for this block's
        # upload from them); the rest are released to the caching host allocator
        pool = self._release_dead()
        main = torch.cuda.current_stream(self.dev)
        self.d2h.wait_stream(main)   # after every kernel that wrote this block
        misses = []
        with torch.cuda.stream(self.d2h):
            for m, kind, n, d in list(_tensor_slots(block)):
                if d.device.type != 'cuda':
                    continue
                h = self._host_of(m, kind, n)
                if dirty or h is None or h.shape != d.shape or h.dtype != d.dtype:
                    if h is None or h.shape != d.shape or h.dtype != d.dtype:
                        self.stats['host_new' if h is None else 'host_retyped'] += 1
                        key = (tuple(d.shape), d.dtype)
                        if pool.get(key):
                            h = pool[key].pop()
                            self.stats['pin_recycled_bytes'] += d.numel() * d.element_size()
                        else:
                            # the next block will most likely need the same: allocated ahead
                            misses.append(key)
                            h = self._take_pinned(d.shape, d.dtype)
                        self.host[(id(m), kind, n)] = (weakref.ref(m), h)
                    h.copy_(d, non_blocking=True)
                    self.stats['d2h_bytes'] += d.numel() * d.element_size()
                d.record_stream(self.d2h)   # HBM reusable only once the copy has run
                _install(m, kind, n, h)
        for m in block.modules():   # plain attributes aliasing a moved buffer (tmp_bias)
            moved = getattr(m, '_lcq_after_move', None)
            if moved is not None:
                moved()
        del pool
        self.resident.discard(i)
        if misses and i + 1 < len(self.blocks):
            self._allocate_ahead(misses)
        self.stats['evict_host_s'] += time.perf_counter() - t_ev

    def _release_dead(self):
        """Drop the host copies of modules that no longer exist; returns those no one else
        holds, by (shape, dtype), for reuse."""
        pool = {}
        for k in [k for k, (ref, _) in self.host.items() if ref() is None]:
            h = self.host.pop(k)[1]
            self.stats['host_released'] += 1
            # exclusive: no other tensor on its storage (the temporary storage object aside)
            # and no other Python reference (the name h and getrefcount's argument aside), so
            # overwriting it is invisible to anyone
            if (torch._C._storage_Use_Count(h.untyped_storage()._cdata) <= 2
                    and sys.getrefcount(h) <= 2):
                pool.setdefault((tuple(h.shape), h.dtype), []).append(h)
            del h
        return pool

    def drain(self):
        self.d2h.synchronize()
        self.h2d.synchronize()
        self.release_ahead()
        self._release_dead()


class Ownership:
    """Which rank materialises what under a sharded plan.

    * ``shard_blocks``: block i belongs to rank i % world (AWQ with quant_out False);
    * ``shard_units``: independent units -- every block linear, a routed expert's linears
      together -- assigned to ranks by LPT on their parameter counts (data-free RTN /
      fake-quant / pack, DeepSeek-V3 experts EP-style). Tensors of a block that are not in
      any unit (norms, the MoE router) and everything outside the blocks stay on every rank.
    Rank-independent and deterministic: every rank computes the same table."""

    def __init__(self, mode: str, rank: int, world: int, block_owner=None, unit_owner=None):
        self.mode, self.rank, self.world = mode, rank, world
        self.block_owner = block_owner or {}
        self.unit_owner = unit_owner or {}

    @classmethod
    def plan(cls, mode, rank, world, model_adapter):
        blocks = model_adapter.get_blocks()
        if mode == 'shard_blocks':
            return cls(mode, rank, world, block_owner={i: i % world for i in range(len(blocks))})
        if mode != 'shard_units':
            raise ValueError(f'no ownership plan for parallel mode {mode}')
        from .parallel import lpt_shard
        # LPT within each block (a block's units are published together, so the block's
        # slowest rank sets its publish time: per-block balance, not only global balance), the
        # ranks rotated by block index so that the per-block leftovers spread over the ranks
        owner = {}
        for bi, block in enumerate(blocks):
            per = {}
            for n, m in model_adapter.get_block_linears(block).items():
                w = getattr(m, 'weight', None)
                per[unit_key(n)] = per.get(unit_key(n), 0) + (w.numel() if w is not None else 0)
            keys = list(per)
            for r, idx in enumerate(lpt_shard([float(per[k]) for k in keys], world)):
                for j in idx:
                    owner[(bi, keys[j])] = (r + bi) % world
        return cls(mode, rank, world, unit_owner=owner)

    def block_of(self, i: int) -> int | None:
        """Owner of the whole block i (shard_blocks), else None."""
        return self.block_owner.get(i)

    def owner_of(self, block_idx: int, linear_name: str) -> int:
        if self.mode == 'shard_blocks':
            return self.block_owner[block_idx]
        return self.unit_owner[(block_idx, unit_key(linear_name))]

    def owns(self, block_idx: int, linear_name: str) -> bool:
        return self.owner_of(block_idx, linear_name) == self.rank

    def owns_block_tensor(self, block_idx: int, rel_name: str, linear_names) -> bool:
        """A tensor of block `block_idx` (name relative to the block): materialised here?"""
        if self.mode == 'shard_blocks':
            return self.block_owner[block_idx] == self.rank
        mod = rel_name.rsplit('.', 1)[0]
        if mod in linear_names:
            return self.owns(block_idx, mod)
        return True
