#!/usr/bin/env python3
"""collective_leg.py — SURVEY §8(d) config D across real GPUs: ncclAllReduce /
ncclReduceScatter of 1 GiB fp32 per rank through libnbxccl's multi-process
communicator (one process per GPU, TCP bootstrap + hipIpc + device flags),
plus the LL128 (1 MiB) and LL (4 KiB) protocols' latency, every output checked.

Run as a CHILD of each bench.py rank (N > 1), so a failure here can never take
the bench's own line down. It is spawned before the parent touches the GPU and
talks over stdin/stdout:

  parent -> child   "ID\\n"               (rank 0 only)
  child  -> parent  "ID <hex> <hex>\\n"   two ncclUniqueIds (direct comm, ring comm)
  parent -> child   "RUN <hex> <hex>\\n"  (every rank, after the parent's broadcast)
  child  -> parent  "RESULT <json>\\n"

Inputs are small integers in fp32 (x_r[i] = (7 i + 13 r) mod 1024), so every
fold order gives the exact sum and the whole output is checked with
torch.equal. Times are per call, measured on this rank; the parent takes the
max over ranks.
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

COUNT = 256 << 20          # fp32 elements per rank: 1 GiB (config D)
LL_COUNT = 1024            # 4 KiB LL AllReduce latency probe
LL128_COUNT = 256 << 10    # 1 MiB LL128 AllReduce (the protocol's largest default message)
LL128_ITERS = 200
WARMUP, ITERS = 2, 5


def _emit(line: str) -> None:
    sys.stdout.write(line + "\n")
    sys.stdout.flush()


def _pkg():
    from __graft_entry__ import _load_package
    nbx = _load_package()
    nbx.load_library()
    return nbx


def _time_calls(fn, iters):
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters


def run(ids, rank, world, dev):
    import torch
    nbx = _pkg()
    torch.cuda.set_device(dev)
    os.environ.pop("NCCL_ALGO", None)
    comm = nbx.Communicator.init_rank(world, nbx.ncclUniqueId.from_buffer_copy(bytes.fromhex(ids[0])), rank)
    os.environ["NCCL_ALGO"] = "Ring"   # read at communicator creation
    comm_ring = nbx.Communicator.init_rank(world, nbx.ncclUniqueId.from_buffer_copy(bytes.fromhex(ids[1])), rank)
    os.environ.pop("NCCL_ALGO", None)
    st = torch.cuda.current_stream().cuda_stream
    F32, SUM = 7, 0
    res = {"rank": rank, "ok": True, "errors": []}

    idx = torch.arange(COUNT, dtype=torch.int32, device="cuda")
    x = ((idx * 7 + 13 * rank) % 1024).to(torch.float32)
    exp = torch.zeros(COUNT, dtype=torch.float32, device="cuda")
    for r in range(world):
        exp += ((idx * 7 + 13 * r) % 1024).to(torch.float32)
    del idx
    y = torch.empty_like(x)

    def check(name, got, want):
        if not torch.equal(got, want):
            res["ok"] = False
            bad = int((got != want).sum().item())
            res["errors"].append(f"{name}: {bad} elements differ")

    for name, c in (("allreduce_direct", comm), ("allreduce_ring", comm_ring)):
        y.zero_()
        c.all_reduce(x.data_ptr(), y.data_ptr(), COUNT, F32, SUM, st)
        torch.cuda.synchronize()
        check(name, y, exp)
        for _ in range(WARMUP):
            c.all_reduce(x.data_ptr(), y.data_ptr(), COUNT, F32, SUM, st)
        res[name + "_ms"] = _time_calls(lambda: c.all_reduce(x.data_ptr(), y.data_ptr(), COUNT, F32, SUM, st), ITERS)

    rc = COUNT // world
    yr = torch.empty(rc, dtype=torch.float32, device="cuda")
    comm.reduce_scatter(x.data_ptr(), yr.data_ptr(), rc, F32, SUM, st)
    torch.cuda.synchronize()
    check("reduce_scatter", yr, exp[rank * rc:(rank + 1) * rc])
    for _ in range(WARMUP):
        comm.reduce_scatter(x.data_ptr(), yr.data_ptr(), rc, F32, SUM, st)
    res["reduce_scatter_ms"] = _time_calls(lambda: comm.reduce_scatter(x.data_ptr(), yr.data_ptr(), rc, F32, SUM, st),
                                           ITERS)

    # LL128 (1 MiB): exact on every one of LL128_ITERS calls with inputs that
    # change per call (a torn 128-byte line or a stale slot would show up as a
    # wrong value), then the per-call latency
    x1 = x[:LL128_COUNT].clone()
    e1 = exp[:LL128_COUNT]
    y1 = torch.empty(LL128_COUNT, dtype=torch.float32, device="cuda")
    bad = 0
    for it in range(LL128_ITERS):
        xi = x1 + float(it % 97)
        comm.all_reduce(xi.data_ptr(), y1.data_ptr(), LL128_COUNT, F32, SUM, st)
        if not torch.equal(y1, e1 + float(world * (it % 97))):
            bad += 1
    torch.cuda.synchronize()
    if bad:
        res["ok"] = False
        res["errors"].append(f"ll128_allreduce: {bad} of {LL128_ITERS} calls wrong")
    res["ll128_checked_calls"] = LL128_ITERS
    res["ll128_allreduce_1MiB_us"] = 1e3 * _time_calls(
        lambda: comm.all_reduce(x1.data_ptr(), y1.data_ptr(), LL128_COUNT, F32, SUM, st), 100)

    xs, ys = x[:LL_COUNT].clone(), torch.empty(LL_COUNT, dtype=torch.float32, device="cuda")
    comm.all_reduce(xs.data_ptr(), ys.data_ptr(), LL_COUNT, F32, SUM, st)
    torch.cuda.synchronize()
    check("ll_allreduce", ys, exp[:LL_COUNT])
    for _ in range(20):
        comm.all_reduce(xs.data_ptr(), ys.data_ptr(), LL_COUNT, F32, SUM, st)
    res["ll_allreduce_4KiB_us"] = 1e3 * _time_calls(
        lambda: comm.all_reduce(xs.data_ptr(), ys.data_ptr(), LL_COUNT, F32, SUM, st), 200)

    torch.cuda.synchronize()
    if comm.async_error() != 0 or comm_ring.async_error() != 0:
        res["ok"] = False
        res["errors"].append("async error")
    comm_ring.destroy()
    comm.destroy()
    return res


def main():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dev = int(os.environ.get("NBX_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    os.environ.setdefault("NBX_TIMEOUT_SEC", "60")
    os.environ.setdefault("NBX_BOOTSTRAP_TIMEOUT", "120")
    if "NBX_BENCH_DEVICE" in os.environ:   # rehearsal: every rank on one GPU, keep LL128 grids co-resident
        os.environ.setdefault("NBX_LL128_MAX_GRID", "32")
    for line in sys.stdin:
        parts = line.split()
        if not parts:
            continue
        if parts[0] == "ID":
            nbx = _pkg()   # imports torch first (one HIP runtime); no GPU use: the root is a host thread
            _emit("ID " + " ".join(bytes(nbx.get_unique_id()).hex() for _ in range(2)))
        elif parts[0] == "RUN":
            try:
                res = run(parts[1:3], rank, world, dev)
            except Exception as e:   # reported to the parent, never raised past it
                res = {"rank": rank, "ok": False, "errors": [f"{type(e).__name__}: {e}"]}
            _emit("RESULT " + json.dumps(res))
            return 0
        elif parts[0] == "QUIT":
            return 0
    return 0


if __name__ == "__main__":
    sys.exit(main())
