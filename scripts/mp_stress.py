#!/usr/bin/env python3
"""mp_stress.py — randomized stress of the multi-process communicator (one
process per rank, every rank on GPU 0): each iteration every rank draws the
same random plan from a shared seed — a sequence of AllReduce /
ReduceScatter / Reduce calls of random datatype, op, size (spanning LL, LL128
one- and two-shot and Simple), stream (two per rank, no caller ordering
between them) and group boundaries (runs of calls inside ncclGroupStart/End,
where runs of compatible LL / LL128 / Simple calls become one launch; a
third of the calls repeat the previous call's kind / type / op so such runs
occur) — issues it without host
synchronisation, then checks every output exactly against torch on the GPU
(small-integer inputs, so every fold order gives the same value; every rank
regenerates every rank's input from the seed). Some AllReduces read the
previous AllReduce's output (same stream): a group run must be cut there. Reports one JSON line per rank
count: iterations, calls, mismatches, first errors.
usage: mp_stress.py [ranks list, default 2,3] [iterations, default 40] [seed]
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# (ncclDataType, torch dtype name); ops: 0 sum, 2 max, 3 min, PREMUL a user
# ncclRedOpCreatePreMulSum with rank r's own scalar (r % 3) + 1 (fp32 / int32 /
# int64 only, where every sum stays exact): expected sum_r s_r * x_r
PREMUL = 9
TYPES = [(7, "float32"), (2, "int32"), (4, "int64"), (6, "float16"), (9, "bfloat16")]
SIZES = [1, 3, 100, 1000, 4099, 16384, 40000, 200000, 1 << 20, 3 << 20]


def plan(rng, n):
    calls = []
    for _ in range(rng.randint(4, 24)):
        kind = rng.choice(["allreduce", "allreduce", "reducescatter", "reduce"])
        dt, tname = rng.choice(TYPES)
        op = rng.choice([0, 0, 2, 3, PREMUL])
        if op == PREMUL and tname not in ("float32", "int32", "int64"):
            op = 0
        root = rng.randrange(n)
        if calls and rng.random() < 0.35:   # runs of one kind / type / op (/ root): what a group launch batches
            p = calls[-1]
            kind, dt, tname, op, root = p["kind"], p["dt"], p["t"], p["op"], p["root"]
        count = rng.choice(SIZES)
        if tname in ("float16", "bfloat16") and op == 0:
            count = min(count, 40000)
        dep = False
        if (calls and calls[-1]["kind"] == "allreduce" and kind == "allreduce" and dt == calls[-1]["dt"] and
                op == calls[-1]["op"] and op != PREMUL and (op in (2, 3) or tname in ("float32", "int32", "int64")) and
                rng.random() < 0.5):
            # reads the previous call's output: a run must be cut before it
            dep, count = True, calls[-1]["count"]
        calls.append({"kind": kind, "dt": dt, "t": tname, "op": op, "count": count, "stream": rng.randint(0, 1),
                      "root": root, "group": rng.random() < 0.5, "dep": dep})
        if dep:   # same stream as the call it reads (a caller orders its own streams)
            calls[-1]["stream"] = calls[-2]["stream"]
    return calls


def _input(torch, c, r, it, k, n, dev):
    total = c["count"] * (n if c["kind"] == "reducescatter" else 1)
    i = torch.arange(total, device=dev, dtype=torch.int64)
    # values small enough that any fold order of n <= 8 sums is exact in fp16 / bf16
    v = (i * 7 + 13 * r + 31 * it + 5 * k) % 16
    return v.to(getattr(torch, c["t"]))


def _describe(torch, c, y, ref, rank, n, settings):
    """mp_diag's description of a wrong output: count, first / last, runs, the
    protocol, the Simple cells, and how many wrong values are zero or equal a
    peer's raw input or the output of the call before (stale data)."""
    from tests import mp_diag
    kind = {"allreduce": "ar", "reducescatter": "rs", "reduce": "red"}[c["kind"]]
    eb = y.element_size()
    raw = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[eb]   # bf16 has no numpy type
    got = y.contiguous().view(raw).cpu().numpy()
    exp = ref.contiguous().view(raw).cpu().numpy()
    geom = None
    proto = mp_diag.proto_of(kind, c["count"], eb, n, settings)
    if proto == "Simple":
        geom = mp_diag.simple_geometry(kind, c["count"], eb, n, settings.get("simpleGrid", 32),
                                       settings.get("sliceBytes", 64 << 10))
    d = mp_diag.describe_mismatch(got, exp, geom, rank * c["count"] if kind == "rs" else 0)
    d["proto"] = proto
    return {"what": mp_diag.format_mismatch(d)}


def rank_main(rank, n, iters, seed, uid, q):
    try:
        import random

        import torch
        from __graft_entry__ import _load_package
        nbx = _load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid), rank)
        from tests import mp_diag
        settings = mp_diag.comm_settings(nbx, comm)
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        bad, ncalls, errs = 0, 0, []
        for it in range(iters):
            rng = random.Random(seed * 1000 + it)
            calls = plan(rng, n)
            live = []
            in_group = False
            torch.cuda.synchronize()
            for k, c in enumerate(calls):
                x = live[-1][3] if c.get("dep") else _input(torch, c, rank, it, k, n, dev)
                y = torch.full((c["count"],), -3, device=dev, dtype=x.dtype)
                torch.cuda.synchronize()
                if c["group"] and not in_group:
                    nbx.group_start()
                    in_group = True
                elif not c["group"] and in_group:
                    nbx.group_end()
                    in_group = False
                s = streams[c["stream"]].cuda_stream
                op = c["op"]
                if op == PREMUL:   # the op's state is copied at enqueue: destroyed right after the call
                    sc = torch.tensor([(rank % 3) + 1], dtype=x.dtype)
                    op = comm.redop_create_premulsum(sc.data_ptr(), c["dt"])
                if c["kind"] == "allreduce":
                    comm.all_reduce(x.data_ptr(), y.data_ptr(), c["count"], c["dt"], op, s)
                elif c["kind"] == "reducescatter":
                    comm.reduce_scatter(x.data_ptr(), y.data_ptr(), c["count"], c["dt"], op, s)
                else:
                    comm.reduce(x.data_ptr(), y.data_ptr() if rank == c["root"] else 0, c["count"], c["dt"], op,
                                c["root"], s)
                if c["op"] == PREMUL:
                    comm.redop_destroy(op)
                live.append((k, c, x, y))   # x too: a queued or in-flight call still reads it
            if in_group:
                nbx.group_end()
            torch.cuda.synchronize()
            refs = []
            for k, c, _x, y in live:
                ncalls += 1
                if c.get("dep"):   # every rank's input is the previous call's (identical) output
                    prev = refs[-1].to(torch.float64)
                    ref = (prev * n if c["op"] == 0 else prev).to(y.dtype)
                else:
                    xs = [_input(torch, c, r, it, k, n, dev) for r in range(n)]
                    st = torch.stack([t.to(torch.float64) for t in xs])
                    if c["op"] == PREMUL:
                        st = st * torch.tensor([(r % 3) + 1 for r in range(n)], dtype=torch.float64,
                                               device=dev).view(-1, 1)
                    ref = st.sum(0) if c["op"] in (0, PREMUL) else (st.amax(0) if c["op"] == 2 else st.amin(0))
                    ref = ref.to(y.dtype)
                refs.append(ref)
                if c["kind"] == "reducescatter":
                    ref = ref[rank * c["count"]:(rank + 1) * c["count"]]
                if c["kind"] == "reduce" and rank != c["root"]:
                    continue
                if not torch.equal(y, ref):
                    bad += 1
                    if len(errs) < 5:   # self-describing (tests/mp_diag.py): where, which cells, what values
                        errs.append({"it": it, "k": k, "call": c, **_describe(torch, c, y, ref, rank, n, settings)})
        ok = comm.async_error() == 0
        comm.destroy()
        q.put((rank, {"calls": ncalls, "mismatches": bad, "errors": errs, "async_ok": ok}))
    except Exception:
        import traceback
        q.put((rank, {"exception": traceback.format_exc()[-2000:]}))


def main():
    ns = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [2, 3]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    os.environ.setdefault("NBX_TIMEOUT_SEC", "60")
    os.environ.setdefault("NBX_BOOTSTRAP_TIMEOUT", "60")
    ctx = mp.get_context("spawn")
    from __graft_entry__ import _load_package
    nbx = _load_package()   # the bootstrap root is a host thread of this process; no GPU use here
    for n in ns:
        uid = bytes(nbx.get_unique_id())
        q = ctx.Queue()
        procs = [ctx.Process(target=rank_main, args=(r, n, iters, seed, uid, q), daemon=True) for r in range(n)]
        for p in procs:
            p.start()
        res = {}
        try:
            for _ in range(n):
                r, out = q.get(timeout=600)
                res[r] = out
        finally:
            for p in procs:
                p.join(30)
                if p.is_alive():
                    p.terminate()
        print(json.dumps({"n": n, "iters": iters, "seed": seed, "ranks": res}), flush=True)


if __name__ == "__main__":
    main()
