"""bench.CollectiveMeter on a world-2 gloo group (CPU): the bytes each rank hands to the
collectives the algorithms call as dist.<op> are counted per op, and the originals are restored
on exit."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, path):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=2)
    try:
        import bench
        orig = dist.all_reduce
        m = bench.CollectiveMeter(2)
        with m:
            t = torch.ones(1024)
            dist.all_reduce(t)
            outs = [torch.empty(256, dtype=torch.float16) for _ in range(2)]
            dist.all_gather(outs, torch.ones(256, dtype=torch.float16))
            dist.broadcast(torch.zeros(100, dtype=torch.int32), src=0)
        torch.save({'per_block': m.per_block(2), 'restored': dist.all_reduce is orig,
                    'sum': t[0].item()}, f'{path}.{rank}')
    finally:
        dist.destroy_process_group()


def test_collective_meter_counts_bytes(tmp_path):
    path = str(tmp_path / 'meter')
    mp.start_processes(_worker, args=(_port(), path), nprocs=2, start_method='spawn')
    for r in range(2):
        res = torch.load(f'{path}.{r}', weights_only=True)
        pb = res['per_block']
        assert res['restored'] and res['sum'] == 2.0
        mb = 2 ** 20
        assert abs(pb['all_reduce'] - round(4096 / 2 / mb, 2)) < 1e-9
        assert pb['calls_per_block'] == 1.5
        total = (4096 + 2 * 512 + 400) / 2 / mb
        assert abs(pb['total'] - round(total, 2)) < 1e-9
    import bench
    assert bench.CollectiveMeter(1).per_block(3) is None
