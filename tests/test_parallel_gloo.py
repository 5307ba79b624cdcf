"""World-size-2 gloo tests (CPU) of the multi-GPU helpers in lightcompress_amd.parallel."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lightcompress_amd import parallel as P


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    finally:
        dist.destroy_process_group()


def run2(fn, world=2):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time
    res, t0 = {}, time.time()
    while len(res) < len(procs):   # a worker that dies fails the test at once, not at timeout
        try:
            r, v = q.get(timeout=1)
            res[r] = v
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead or time.time() - t0 > 240:
                for p in procs:
                    p.kill()
                raise AssertionError(f'worker exit codes {[p.exitcode for p in procs]}')
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _mean(rank, world):
    t = torch.full((3,), float(rank + 1))
    P.allreduce_mean_(t)
    return t.tolist()


def _pick(rank, world):
    # rank 1 has the smaller loss -> its scales win everywhere
    scales = torch.full((4,), float(rank + 10))
    return P.awq_pick_best(0.5 - 0.1 * rank, scales).tolist()


def _pick_tie(rank, world):
    scales = torch.full((2,), float(rank))
    return P.awq_pick_best(0.25, scales).tolist()  # tie -> highest rank (MAX reduce)


def _gather(rank, world):
    rows = 7
    s, e = P.row_shard(rows, rank, world)
    local = torch.arange(rows * 3, dtype=torch.float32).reshape(rows, 3)[s:e]
    return P.gather_rows(local, rows).tolist()


def _bcast(rank, world):
    m = torch.nn.Linear(4, 2)
    with torch.no_grad():
        m.weight.fill_(rank)
        m.bias.fill_(rank)
    P.broadcast_block(m, owner=1)
    return [m.weight.sum().item(), m.bias.sum().item()]


def _bcast_owner_buffers(rank, world):
    # the owner's transform registered static act qparams the other rank does not have
    blk = torch.nn.Sequential(torch.nn.Linear(4, 2), torch.nn.Linear(2, 2))
    blk[0].register_buffer('buf_scales', torch.full((2, 1), float(rank)))
    if rank == 1:
        blk[0].register_buffer('buf_act_scales_0', torch.tensor(0.125))
        blk[1].register_buffer('buf_act_zeros_0', torch.tensor(3.0, dtype=torch.bfloat16))
    P.broadcast_block(blk, owner=1)
    return [blk[0].buf_scales.sum().item(), blk[0].buf_act_scales_0.item(),
            str(blk[1].buf_act_zeros_0.dtype), blk[1].buf_act_zeros_0.item()]


def test_allreduce_mean():
    res = run2(_mean)
    assert res[0] == res[1] == [1.5, 1.5, 1.5]


def test_awq_pick_best():
    res = run2(_pick)
    assert res[0] == res[1] == [11.0] * 4


def test_awq_pick_best_tie():
    res = run2(_pick_tie)
    assert res[0] == res[1] == [1.0, 1.0]


def test_gather_rows():
    res = run2(_gather)
    ref = torch.arange(21, dtype=torch.float32).reshape(7, 3).tolist()
    assert res[0] == res[1] == ref


def test_broadcast_block():
    res = run2(_bcast)
    assert res[0] == res[1] == [8.0, 2.0]


@pytest.mark.parametrize('world', [1, 2, 3, 8])
def test_shards_cover_exactly_once(world):
    n = 32
    owned = sorted(i for r in range(world) for i in P.block_shard(n, r, world))
    assert owned == list(range(n))
    costs = [float((i * 7) % 5 + 1) for i in range(25)]
    parts = P.lpt_shard(costs, world)
    assert sorted(i for p in parts for i in p) == list(range(25))
    loads = [sum(costs[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(costs)
    spans = [P.row_shard(1000, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == 1000
    assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def test_broadcast_block_creates_owner_only_buffers():
    res = run2(_bcast_owner_buffers)
    assert res[0] == res[1] == [2.0, 0.125, 'torch.bfloat16', 3.0]
