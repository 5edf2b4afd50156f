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


STUB_CHILD = r'''
import json, os, sys
rank = int(os.environ["RANK"])
mode = os.environ.get("STUB_MODE", "ok")
for line in sys.stdin:
    p = line.split()
    if p and p[0] == "ID":
        print("ID aa bb", flush=True)
    elif p and p[0] == "RUN":
        assert p[1:3] == ["aa", "bb"]
        if mode == "die" and rank == 1:
            sys.exit(3)
        if mode == "hang" and rank == 1:
            import time; time.sleep(600)
        print("RESULT " + json.dumps({"rank": rank, "ok": True, "errors": [],
              "allreduce_direct_ms": 10.0 + rank, "allreduce_ring_ms": 20.0 + rank,
              "reduce_scatter_ms": 5.0 + rank, "ll_allreduce_4KiB_us": 7.0 + rank,
              "sweep_bytes": [4096, 65536], "sweep_LL_us": [3.0 + rank, 9.0 - rank],
              "sweep_LL128_us": [4.0, 5.0], "sweep_LL128_oneshot_us": [4.5, 5.5],
              "sweep_Simple_us": [50.0, 60.0 + rank]}), flush=True)
        break
'''


def _leg_worker(rank, world, port, script, mode, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      STUB_MODE=mode)
    import bench
    child = bench._spawn_collective_leg(world, script)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = bench.collective_leg(child, world, rank, result_timeout=10.0)
    q.put((rank, out, child.returncode))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["ok", "die", "hang"])
def test_collective_leg_protocol_gloo(tmp_path, mode):
    """bench.py's config-D leg: the parent <-> child protocol, the id broadcast,
    max-over-ranks aggregation (algbw / busbw), and that a child that dies or
    hangs is reported (ok: false) without hanging or failing the bench."""
    script = tmp_path / "stub_child.py"
    script.write_text(STUB_CHILD)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_leg_worker, args=(r, world, port, str(script), mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (o, rc)) for r, o, rc in [q.get(timeout=180) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out = res[0][0]
    assert res[1][0] is None
    S = (256 << 20) * 4
    if mode == "ok":
        assert out["ok"] is True and "errors" not in out
        assert out["allreduce_direct"]["ms"] == 11.0          # max over ranks
        alg = S / 11e-3 / 1e9
        assert abs(out["allreduce_direct"]["algbw_GBs"] - round(alg, 2)) < 1e-9
        assert abs(out["allreduce_direct"]["busbw_GBs"] - round(alg * 2 * (world - 1) / world, 2)) < 1e-9
        assert out["reduce_scatter"]["ms"] == 6.0
        assert abs(out["reduce_scatter"]["busbw_GBs"] - round(S / 6e-3 / 1e9 * (world - 1) / world, 2)) < 1e-9
        assert out["ll_allreduce_4KiB_us"] == 8.0
        sw = out["protocol_sweep"]   # column-wise max over ranks
        assert sw["bytes"] == [4096, 65536]
        assert sw["LL"] == [4.0, 9.0] and sw["LL128"] == [4.0, 5.0] and sw["Simple"] == [50.0, 61.0]
        assert sw["LL128_oneshot"] == [4.5, 5.5]
    else:
        assert out["ok"] is False
        assert any(e.startswith("rank 1:") for e in out["errors"])
        assert out["allreduce_direct"] is None


STUB_CLIQUE = r'''
import json, os, sys
mode = os.environ.get("STUB_MODE", "ok")
for line in sys.stdin:
    p = line.split()
    if p and p[0] == "RUN":
        n, devs = int(p[1]), [int(d) for d in p[2].split(",")]
        if mode == "die":
            sys.exit(3)
        print("RESULT " + json.dumps({"ok": True, "errors": [], "n_ranks": n, "devices": devs,
                                      "allreduce_ms": 8.0, "reduce_scatter_ms": 4.0}), flush=True)
        break
'''


def _clique_worker(rank, world, port, script, mode, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      STUB_MODE=mode)
    import bench
    child = bench._spawn_clique_leg(world, rank, script)
    assert (child is None) == (rank != 0)   # rank 0 alone runs the single-process clique
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = bench.clique_leg(child, world, rank, dev=3 + rank, result_timeout=10.0)
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["ok", "die"])
def test_clique_leg_protocol_gloo(tmp_path, mode):
    """bench.py's single-process (ncclCommInitAll) config-D leg: rank 0's child
    gets every rank's device, the other ranks wait on the host store and
    return None, algbw / busbw are derived, and a dying child is reported."""
    script = tmp_path / "stub_clique.py"
    script.write_text(STUB_CLIQUE)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_clique_worker, args=(r, world, port, str(script), mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] is None
    out = res[0]
    if mode == "ok":
        assert out["ok"] is True and out["devices"] == [3, 4]
        S = (256 << 20) * 4
        assert out["allreduce"]["ms"] == 8.0
        assert abs(out["allreduce"]["busbw_GBs"] - round(S / 8e-3 / 1e9 * 2 * (world - 1) / world, 2)) < 1e-9
        assert abs(out["reduce_scatter"]["busbw_GBs"] - round(S / 4e-3 / 1e9 * (world - 1) / world, 2)) < 1e-9
    else:
        assert out["ok"] is False and out["errors"][0].startswith("no result from the clique leg")
