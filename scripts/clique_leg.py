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


def run(n: int, devs: list, count: int = COUNT) -> dict:
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    nbx.load_library()
    F32, SUM = 7, 0
    res = {"ok": True, "errors": [], "n_ranks": n, "devices": devs}
    comms = nbx.Communicator.init_all(devs)
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
    for c in comms:
        c.destroy()
    return res


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
