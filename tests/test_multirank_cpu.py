"""World-size-2 gloo tests (CPU) of the multi-GPU bench harness: the barrier
and max-over-ranks timing that bench.py uses for N > 1, and the weak-scaling
aggregation (value = N x bytes / max time)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    bench._barrier(world)
    t = 1.0 + rank          # rank r "took" 1 + r seconds
    m = bench.max_over_ranks(t, world)
    value = world * bench.ALG_BYTES / (m / 10) / 2**30
    q.put((rank, m, value))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_max_over_ranks_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, m, value in res:
        assert m == float(world)   # max over ranks of 1 + r
        assert abs(value - world * 2.25 / (world / 10)) < 1e-9
