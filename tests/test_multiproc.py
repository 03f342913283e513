"""Multi-GPU path logic on CPU: shard ranges, and the bench's barrier +
max-over-ranks timing over a world_size-2 gloo group (no data-path collective)."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from fedtree_amd.multi import shard_range


@pytest.mark.parametrize("total,world", [(0, 1), (1, 2), (10, 3), (20_000_000, 8), (80_000_000, 8), (7, 8)])
def test_shard_range_partitions(total, world):
    spans = [shard_range(total, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(20_000_000, rank, world)
    dist.barrier()
    elapsed = torch.tensor([1.0 + rank], dtype=torch.float64)     # rank 1 is the slow one
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    units = torch.tensor([hi - lo], dtype=torch.int64)
    dist.all_reduce(units)
    q.put((rank, lo, hi, float(elapsed.item()), int(units.item())))
    dist.destroy_process_group()


def test_gloo_world2_barrier_and_max_timing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert [r[1:3] for r in res] == [(0, 10_000_000), (10_000_000, 20_000_000)]
    assert all(r[3] == 2.0 for r in res)          # value uses the slowest rank's time
    assert all(r[4] == 20_000_000 for r in res)    # shards cover the job exactly
