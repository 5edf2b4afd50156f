#!/usr/bin/env python3
"""clique_leg.py — SURVEY §8(d) config D through the SINGLE-process
communicator: ncclCommInitAll over all N GPUs of the bench (init.cc:1678-1734),
no IPC, no bootstrap, one thread issuing every rank's call inside
ncclGroupStart/End (nccl.h.in:387-407). Run next to collective_leg.py (the
one-process-per-GPU communicator) so that on a multi-GPU node a failure of the
multi-process plumbing can be told apart from a failure of the xGMI data path
(VERDICT r2 item 6).

Spawned by bench.py rank 0 before it touches the GPU, idle until told:
  parent -> child   "RUN <n> <dev0,dev1,...>\\n"
  child  -> parent  "RESULT <json>\\n"
Inputs are small integers in fp32 (x_r[i] = (7 i + 13 r) mod 1024), so every
fold order gives the exact sum and every rank's whole output is checked.
Then 4 KiB / 64 KiB / 1 MiB AllReduces (the in-kernel LL / LL128 transport when
the devices are distinct), each checked and timed per call. Config D runs in-kernel
(distinct devices: the Simple kernels over staging, forced for every size with
NBX_CLIQUE_SIMPLE_MAX_BYTES), then again on a second clique with
NBX_CLIQUE_SIMPLE=0 (the event-ordered direct fold that reads peers' buffers in
place) — `fold_*` — so the driver's multi-GPU run measures both data paths
over xGMI (the clique's default switches from the first to the second above
32 MiB).
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

COUNT = 256 << 20   # fp32 elements per rank: 1 GiB (config D)
WARMUP, ITERS = 2, 5
SMALL_BYTES, SMALL_ITERS = (4096, 65536, 1 << 20), 100   # then LL / LL128 latency, one thread driving every rank
os.environ.setdefault("NBX_TIMEOUT_SEC", "30")   # before the library loads: a stuck wait ends the probe, not the bench


def run(n: int, devs: list, count: int = COUNT) -> dict:
    import ctypes

    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    lib = nbx.load_library()
    F32, SUM = 7, 0
    res = {"ok": True, "errors": [], "n_ranks": n, "devices": devs}
    # config D in-kernel whatever its size (the default hands messages above
    # NBX_CLIQUE_SIMPLE_MAX_BYTES to the fold), then on the fold below
    os.environ["NBX_CLIQUE_SIMPLE_MAX_BYTES"] = str(1 << 62)
    try:
        comms = nbx.Communicator.init_all(devs)
    finally:
        os.environ.pop("NBX_CLIQUE_SIMPLE_MAX_BYTES", None)
    vals = (ctypes.c_int64 * 9)()
    res["simple_in_kernel"] = lib.nbxDebugCommSettings(comms[0].handle, vals, 9) == 9 and vals[4] > 0
    xs, ys, rs, streams, exps = [], [], [], [], []
    rc = count // n
    for r, d in enumerate(devs):
        with torch.cuda.device(d):
            idx = torch.arange(count, dtype=torch.int32, device=f"cuda:{d}")
            xs.append(((idx * 7 + 13 * r) % 1024).to(torch.float32))
            e = torch.zeros(count, dtype=torch.float32, device=f"cuda:{d}")
            for q in range(n):
                e += ((idx * 7 + 13 * q) % 1024).to(torch.float32)
            del idx
            exps.append(e)
            ys.append(torch.full((count,), -1.0, device=f"cuda:{d}"))
            rs.append(torch.full((rc,), -1.0, device=f"cuda:{d}"))
            streams.append(torch.cuda.Stream(device=d))

    def sync():
        for d in devs:
            torch.cuda.synchronize(d)

    # the inputs and the -1 sentinels are written on each device's current
    # stream; the collectives run on streams[r]: finish the former first (the
    # N = 4 rehearsal r3k saw every element differ: the sentinel fill landed
    # after the collective's output)
    sync()
    def allreduce():
        nbx.group_start()
        for r in range(n):
            comms[r].all_reduce(xs[r].data_ptr(), ys[r].data_ptr(), count, F32, SUM, streams[r].cuda_stream)
        nbx.group_end()

    def reduce_scatter():
        nbx.group_start()
        for r in range(n):
            comms[r].reduce_scatter(xs[r].data_ptr(), rs[r].data_ptr(), rc, F32, SUM, streams[r].cuda_stream)
        nbx.group_end()

    def timed(fn):
        for _ in range(WARMUP):
            fn()
        sync()
        t0 = time.perf_counter()
        for _ in range(ITERS):
            fn()
        sync()
        return (time.perf_counter() - t0) * 1e3 / ITERS

    allreduce()
    sync()
    for r in range(n):
        if not torch.equal(ys[r], exps[r]):
            res["ok"] = False
            res["errors"].append(f"allreduce rank {r}: {int((ys[r] != exps[r]).sum())} elements differ")
    res["allreduce_ms"] = timed(allreduce)
    reduce_scatter()
    sync()
    for r in range(n):
        want = exps[r][r * rc:(r + 1) * rc]
        if not torch.equal(rs[r], want):
            res["ok"] = False
            res["errors"].append(f"reduce_scatter rank {r}: {int((rs[r] != want).sum())} elements differ")
    res["reduce_scatter_ms"] = timed(reduce_scatter)
    small_calls(nbx, torch, comms, xs, ys, exps, streams, sync, res)
    for c in comms:
        c.destroy()
    # the same config D on the event-ordered fold path (a second clique)
    os.environ["NBX_CLIQUE_SIMPLE"] = "0"
    try:
        comms = nbx.Communicator.init_all(devs)
    finally:
        os.environ.pop("NBX_CLIQUE_SIMPLE", None)
    for r in range(n):
        with torch.cuda.device(ys[r].device):
            ys[r].fill_(-1.0)
            rs[r].fill_(-1.0)
    sync()
    allreduce()
    reduce_scatter()
    sync()
    for r in range(n):
        if not torch.equal(ys[r], exps[r]) or not torch.equal(rs[r], exps[r][r * rc:(r + 1) * rc]):
            res["ok"] = False
            res["errors"].append(f"fold path rank {r}: output differs")
    res["fold_allreduce_ms"] = timed(allreduce)
    res["fold_reduce_scatter_ms"] = timed(reduce_scatter)
    for c in comms:
        c.destroy()
    return res


def small_calls(nbx, torch, comms, xs, ys, exps, streams, sync, res):
    """LL / LL128-sized AllReduces (in-kernel when the clique's devices are
    distinct, cliqueInitTransport): each size checked exactly against a -1
    sentinel, then timed; the first device error ends the probe (a stuck wait
    gives up after NBX_TIMEOUT_SEC, set low for this child)."""
    import ctypes
    lib = nbx.load_library()
    lib.nbxDebugCommProtoMask.argtypes = [ctypes.c_void_p]
    lib.nbxDebugCommProtoMask.restype = ctypes.c_int
    n = len(comms)
    res["small_in_kernel"] = all(lib.nbxDebugCommProtoMask(c.handle) >= 0 for c in comms)
    us = {}
    for nbytes in SMALL_BYTES:
        cnt = nbytes // 4

        def ar():
            nbx.group_start()
            for r in range(n):
                comms[r].all_reduce(xs[r].data_ptr(), ys[r].data_ptr(), cnt, 7, 0, streams[r].cuda_stream)
            nbx.group_end()

        for r in range(n):
            with torch.cuda.device(ys[r].device):
                ys[r][:cnt].fill_(-1.0)
        sync()
        ar()
        sync()
        if any(c.async_error() != 0 for c in comms):
            res["ok"] = False
            res["errors"].append(f"small allreduce {nbytes} B: device wait gave up")
            break
        wrong = [r for r in range(n) if not torch.equal(ys[r][:cnt], exps[r][:cnt])]
        if wrong:
            res["ok"] = False
            res["errors"].append(f"small allreduce {nbytes} B: ranks {wrong} differ")
            break
        for _ in range(10):
            ar()
        sync()
        t0 = time.perf_counter()
        for _ in range(SMALL_ITERS):
            ar()
        sync()
        us[str(nbytes)] = round((time.perf_counter() - t0) * 1e6 / SMALL_ITERS, 2)
    res["allreduce_small_us_per_call"] = us


def main():
    for line in sys.stdin:
        parts = line.split()
        if not parts:
            continue
        if parts[0] == "RUN":
            try:
                n = int(parts[1])
                devs = [int(d) for d in parts[2].split(",")]
                res = run(n, devs)
            except Exception as e:   # reported to the parent, never raised past it
                res = {"ok": False, "errors": [f"{type(e).__name__}: {e}"]}
            sys.stdout.write("RESULT " + json.dumps(res) + "\n")
            sys.stdout.flush()
            return 0
        if parts[0] == "QUIT":
            return 0
    return 0


if __name__ == "__main__":
    sys.exit(main())
