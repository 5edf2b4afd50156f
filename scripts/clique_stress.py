#!/usr/bin/env python3
"""clique_stress.py — randomized, exact-checked stress of the in-process
clique (ncclCommInitAll, one thread driving every rank) with its in-kernel LL /
LL128 transport forced on for ranks that share the one GPU of the test box
(NBX_CLIQUE_LL=1; each rank's kernel waits for its peers', so every rank has
its own streams, and GPU_MAX_HW_QUEUES gives every stream its own hardware
queue — set here, before anything loads HIP). Same plans as mp_stress.py
(AllReduce / ReduceScatter / Reduce, random dtype, op — user PreMulSum with
per-rank scalars included — size across LL, LL128
one- and two-shot and the Simple-sized fold path, groups), plus stream switches
and calls whose ranks all share one stream (those take the fold path), so the
ordering between the two paths is exercised too.
Then, with --perf, times back-to-back 4 KiB fp32 AllReduces per call.
Prints one JSON line per rank count.

The rig needs one hardware queue per stream: with ranks sharing one GPU, a
rank's kernel queued behind a waiting peer's kernel on a shared hardware queue
never starts, and every rank's device wait times out. Each rank count creates
n x streams + 1 streams and they are not returned, so the rank counts of one
process must fit GPU_MAX_HW_QUEUES together (24 here by default,
NBX_STRESS_HW_QUEUES up to 32): profiles/r6/clique_queues_r6x/ — 2,3,4,8 in
one process (30 streams) times out at 24 queues and is exact at 32; 8,8,8 (27)
times out at its third 8 at 24. The script refuses such a list up front.
usage: clique_stress.py ranks_list iterations seed [--perf]
"""
from __future__ import annotations

import json
import os
import sys
import time

# assigned, not defaulted: the GPU box exports GPU_MAX_HW_QUEUES=4, and with fewer hardware
# queues than streams one rank's kernel can queue behind a peer's waiting one
os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, int(os.environ.get("NBX_STRESS_HW_QUEUES", "24"))))
os.environ.setdefault("NBX_CLIQUE_LL", "1")
os.environ.setdefault("NBX_TIMEOUT_SEC", "5")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

from mp_stress import PREMUL, _input, plan  # noqa: E402


def run(n: int, iters: int, seed: int, perf: bool) -> dict:
    import ctypes
    import random

    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    lib = nbx.load_library()
    lib.nbxDebugCommProtoMask.argtypes = [ctypes.c_void_p]
    lib.nbxDebugCommProtoMask.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    comms = nbx.Communicator.init_all([0] * n)
    in_kernel = all(lib.nbxDebugCommProtoMask(c.handle) >= 0 for c in comms)
    nstreams = 2 if n <= 4 else 1
    streams = [[torch.cuda.Stream() for _ in range(nstreams)] for _ in range(n)]
    shared = torch.cuda.Stream()
    bad, ncalls, errs = 0, 0, []
    for it in range(iters):
        rng = random.Random(seed * 1000 + it)
        calls = plan(rng, n)
        for c in calls:
            c["shared"] = rng.random() < 0.2
            c["stream"] = c["stream"] % nstreams
        live = []
        in_group = False
        torch.cuda.synchronize()
        for k, c in enumerate(calls):
            xs = [_input(torch, c, r, it, k, n, dev) for r in range(n)]
            ys = [torch.full((c["count"],), -3, device=dev, dtype=xs[0].dtype) for _ in range(n)]
            torch.cuda.synchronize()
            if c["group"] and not in_group:
                nbx.group_start()
                in_group = True
            elif not c["group"] and in_group:
                nbx.group_end()
                in_group = False
            if not in_group:   # one thread drives every rank: their calls of one collective form a group
                nbx.group_start()
            for r in range(n):
                s = (shared if c["shared"] else streams[r][c["stream"]]).cuda_stream
                op = c["op"]
                if op == PREMUL:   # rank r's own scalar (r % 3) + 1; state copied at enqueue
                    sc = torch.tensor([(r % 3) + 1], dtype=xs[r].dtype)
                    op = comms[r].redop_create_premulsum(sc.data_ptr(), c["dt"])
                if c["kind"] == "allreduce":
                    comms[r].all_reduce(xs[r].data_ptr(), ys[r].data_ptr(), c["count"], c["dt"], op, s)
                elif c["kind"] == "reducescatter":
                    comms[r].reduce_scatter(xs[r].data_ptr(), ys[r].data_ptr(), c["count"], c["dt"], op, s)
                else:
                    comms[r].reduce(xs[r].data_ptr(), ys[r].data_ptr() if r == c["root"] else 0, c["count"],
                                    c["dt"], op, c["root"], s)
                if c["op"] == PREMUL:
                    comms[r].redop_destroy(op)
            if not in_group:
                nbx.group_end()
            live.append((k, c, xs, ys))
        if in_group:
            nbx.group_end()
        torch.cuda.synchronize()
        errs_now = [c.async_error() for c in comms]
        print(f"# n={n} it={it} calls={len(calls)} async={errs_now} t={time.strftime('%X')}", file=sys.stderr,
              flush=True)
        if any(errs_now):   # a device wait gave up: later calls would each wait out the timeout too
            out = {"n": n, "iters": it + 1, "seed": seed, "in_kernel": in_kernel, "checked": ncalls,
                   "mismatches": bad, "errors": errs, "async_ok": False,
                   "last_error": (lib.ncclGetLastError(None) or b"").decode(errors="replace")}
            for c in comms:
                c.destroy()
            return out
        for k, c, xs, ys in live:
            st = torch.stack([t.to(torch.float64) for t in xs])
            if c["op"] == PREMUL:
                st = st * torch.tensor([(r % 3) + 1 for r in range(n)], dtype=torch.float64, device=dev).view(-1, 1)
            ref = st.sum(0) if c["op"] in (0, PREMUL) else (st.amax(0) if c["op"] == 2 else st.amin(0))
            ref = ref.to(ys[0].dtype)
            for r in range(n):
                if c["kind"] == "reduce" and r != c["root"]:
                    continue
                want = ref[r * c["count"]:(r + 1) * c["count"]] if c["kind"] == "reducescatter" else ref
                ncalls += 1
                if not torch.equal(ys[r], want):
                    bad += 1
                    if len(errs) < 5:
                        errs.append({"it": it, "k": k, "rank": r, "call": c, "wrong": int((ys[r] != want).sum())})
    out = {"n": n, "iters": iters, "seed": seed, "in_kernel": in_kernel, "checked": ncalls, "mismatches": bad,
           "errors": errs}
    if perf:
        count = 1024
        xs = [torch.ones(count, device=dev) for _ in range(n)]
        ys = [torch.zeros(count, device=dev) for _ in range(n)]

        def one():
            nbx.group_start()
            for r in range(n):
                comms[r].all_reduce(xs[r].data_ptr(), ys[r].data_ptr(), count, 7, 0, streams[r][0].cuda_stream)
            nbx.group_end()

        for _ in range(20):
            one()
        torch.cuda.synchronize()
        reps = 200
        t0 = time.perf_counter()
        for _ in range(reps):
            one()
        torch.cuda.synchronize()
        out["allreduce_4KiB_us_per_call"] = round((time.perf_counter() - t0) * 1e6 / reps, 2)
        out["perf_exact"] = all(bool(torch.all(y == n)) for y in ys)
    out["async_ok"] = all(c.async_error() == 0 for c in comms)
    for c in comms:
        c.destroy()
    return out


def streams_needed(ns) -> int:
    """Streams run() creates over the rank counts `ns` in one process."""
    return sum(n * (2 if n <= 4 else 1) + 1 for n in ns)


def main():
    ns = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [2, 3]
    queues = int(os.environ["GPU_MAX_HW_QUEUES"])
    if streams_needed(ns) > queues:
        sys.exit(f"clique_stress: rank counts {ns} need {streams_needed(ns)} streams in one process, more than the "
                 f"{queues} hardware queues (GPU_MAX_HW_QUEUES): run them in separate processes")
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    perf = "--perf" in sys.argv
    for n in ns:
        print(json.dumps(run(n, iters, seed, perf)), flush=True)


if __name__ == "__main__":
    main()
