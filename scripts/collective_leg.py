#!/usr/bin/env python3
"""collective_leg.py — SURVEY §8(d) config D across real GPUs: ncclAllReduce /
ncclReduceScatter of 1 GiB fp32 per rank through libnbxccl's multi-process
communicator (one process per GPU, TCP bootstrap + hipIpc + device flags),
plus the LL128 (1 MiB) and LL (4 KiB) protocols' latency and config E (int64
max + fp8 sum AllReduce, 128 MiB), every output checked.

Run as a CHILD of each bench.py rank (N > 1), so a failure here can never take
the bench's own line down. It is spawned before the parent touches the GPU and
talks over stdin/stdout:

  parent -> child   "ID\\n"               (rank 0 only)
  child  -> parent  "ID <hex> x9\\n"      ncclUniqueIds: direct, ring, the LL / LL128 /
                                         LL128-one-shot / Simple comms of the protocol
                                         sweep, and the three Simple-knob comms
  parent -> child   "RUN <hex> x9\\n"     (every rank, after the parent's broadcast)
  child  -> parent  "PARTIAL <json>\\n"    (after every stage: the results so far; the
                                         parent reports the last one if the leg runs out
                                         of its time budget)
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
SIMPLE_STRESS_COUNT = 8 << 20   # 32 MiB fp32: above every LL/LL128 threshold
SIMPLE_STRESS_ITERS = 30
E_I64 = 16 << 20           # config E: int64 elements (128 MiB)
E_F8 = 128 << 20           # config E: fp8 elements (128 MiB)
WARMUP, ITERS = 2, 5


def _emit(line: str) -> None:
    sys.stdout.write(line + "\n")
    sys.stdout.flush()


def _progress(msg: str, res: dict | None = None) -> None:
    """To this rank's leg log (stderr; its tail is reported on failure) and,
    with `res`, the results so far to the parent (a PARTIAL line)."""
    sys.stderr.write(f"[leg {time.strftime('%H:%M:%S')}] {msg}\n")
    sys.stderr.flush()
    if res is not None:
        _emit("PARTIAL " + json.dumps(dict(res, stage=msg)))


def _ipc_repairs(lib, comm) -> int | None:
    """Connection buffers this communicator re-exported at creation because a
    peer's IPC mapping of them showed other memory (nbxDebugCommSettings[8])."""
    import ctypes
    vals = (ctypes.c_int64 * 10)()
    return int(vals[8]) if lib.nbxDebugCommSettings(comm.handle, vals, 10) >= 9 else None


def _pkg():
    from __graft_entry__ import _load_package
    nbx = _load_package()
    nbx.load_library()
    return nbx


_ALIGN = []   # set by run(): a tiny collective that lines the ranks up before a timed loop


def _time_calls(fn, iters, warmup=2):
    """ms per call of `fn` after `warmup` untimed calls, started with the ranks
    lined up (a small AllReduce + device sync), so no rank's timed loop absorbs
    a peer's late arrival."""
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    for f in _ALIGN:
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters


SWEEP_BYTES = [4 << 10, 32 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20]
SWEEP_PROTOS = (("LL", {"NCCL_PROTO": "LL", "NBX_LL_MAX_BYTES": str(16 << 20)}),
                ("LL128", {"NCCL_PROTO": "LL128", "NBX_LL128_MAX_BYTES": str(16 << 20)}),
                ("LL128_oneshot", {"NCCL_PROTO": "LL128", "NBX_LL128_MAX_BYTES": str(16 << 20),
                                   "NBX_LL128_ONESHOT_MAX": str(16 << 20)}),
                ("Simple", {"NCCL_PROTO": "Simple"}))


def protocol_sweep(ids, rank, world, st, shared_gpu, res):
    """AllReduce fp32 sum latency per protocol and message size (one
    communicator per protocol, forced by NCCL_PROTO at init, the LL / LL128
    buffers enlarged to 16 MiB; "LL128" switches to the two-shot kernel above
    256 KiB with > 2 ranks, "LL128_oneshot" never does), each size checked
    exactly once."""
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    sizes = [b for b in SWEEP_BYTES if not shared_gpu or b <= (1 << 20)]
    res["sweep_bytes"] = sizes
    for (name, env), uid in zip(SWEEP_PROTOS, ids):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            c = nbx.Communicator.init_rank(world, nbx.ncclUniqueId.from_buffer_copy(bytes.fromhex(uid)), rank)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        times = []
        for b in sizes:
            n = b // 4
            idx = torch.arange(n, dtype=torch.int32, device="cuda")
            x = ((idx * 5 + 3 * rank) % 512).to(torch.float32)
            want = sum(((idx * 5 + 3 * r) % 512).to(torch.float32) for r in range(world))
            y = torch.full_like(x, -1.0)   # sentinel: an element nobody wrote stays -1
            c.all_reduce(x.data_ptr(), y.data_ptr(), n, 7, 0, st)
            torch.cuda.synchronize()
            if not torch.equal(y, want):
                res["ok"] = False
                bad = (y != want).nonzero().flatten()
                i0, i1 = int(bad[0]), int(bad[-1])
                own = ((idx * 5 + 3 * rank) % 512).to(torch.float32)
                res["errors"].append(
                    f"sweep {name} {b} B: output differs at {bad.numel()} of {n} elements [{i0}, {i1}] "
                    f"(got {float(y[i0])} want {float(want[i0])}; unwritten {int((y[bad] == -1.0).sum())}, "
                    f"equal to this rank's input {int((y[bad] == own[bad]).sum())})")
            iters = 50 if b <= (1 << 20) else 20
            for _ in range(5):
                c.all_reduce(x.data_ptr(), y.data_ptr(), n, 7, 0, st)
            times.append(round(1e3 * _time_calls(lambda: c.all_reduce(x.data_ptr(), y.data_ptr(), n, 7, 0, st),
                                                 iters), 2))
        res["sweep_" + name + "_us"] = times
        if name == "LL128":
            ll128_stress(c, rank, world, st, res)
        if c.async_error() != 0:
            res["ok"] = False
            res["errors"].append(f"sweep {name}: async error")
        c.destroy()


# the Simple transport's init-time knobs against the default (64 KiB slices,
# 128 workgroups, 2 slots), on config D's 1 GiB direct AllReduce: what
# scripts/set_thresholds.py reads to pick the xGMI defaults from a node run
SIMPLE_KNOBS = (("slice256K", {"NBX_SIMPLE_SLICE_BYTES": str(256 << 10)}),
                ("grid64", {"NBX_SIMPLE_MAX_GRID": "64"}),
                ("slots4", {"NBX_SIMPLE_SLOTS": "4"}))


def simple_knob_sweep(ids, rank, world, st, x, y, exp, res):
    """1 GiB AllReduce ms per Simple knob setting (one communicator each, the
    knob set at creation; every rank sets the same), each output checked."""
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    out = {}
    for (name, env), uid in zip(SIMPLE_KNOBS, ids):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            c = nbx.Communicator.init_rank(world, nbx.ncclUniqueId.from_buffer_copy(bytes.fromhex(uid)), rank)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        y.zero_()
        c.all_reduce(x.data_ptr(), y.data_ptr(), COUNT, 7, 0, st)
        torch.cuda.synchronize()
        if not torch.equal(y, exp):
            res["ok"] = False
            res["errors"].append(f"simple knob {name}: {int((y != exp).sum().item())} elements differ")
        out[name] = _time_calls(lambda: c.all_reduce(x.data_ptr(), y.data_ptr(), COUNT, 7, 0, st), ITERS)
        if c.async_error() != 0:
            res["ok"] = False
            res["errors"].append(f"simple knob {name}: async error")
        c.destroy()
    res["simple_knobs_ms"] = out


CURVE_BYTES = (64 << 20, 256 << 20)   # = bench.CURVE_BYTES

LL128_STRESS_CALLS = 1000   # per size: one-shot and (n > 2) two-shot -> >= 2000 calls


def ll128_stress(c, rank, world, st, res):
    """The 64-byte LL128 line across the fabric (LL128 is off by
    default across GPUs until a node run shows it whole): LL128_STRESS_CALLS
    AllReduces per size on the NCCL_PROTO=LL128 communicator (LL128 forced, its
    creation-time probe passed), inputs changing every call, every output
    compared exactly on the GPU. Sizes: 96 KiB (one-shot) and, with more than 2
    ranks, 1 MiB (two-shot above the 256 KiB one-shot limit); at 2 ranks 1 MiB
    is one-shot too. A torn line would show as a wrong element."""
    import torch
    calls = bad = 0
    sizes = {"oneshot": 24 << 10, "twoshot" if world > 2 else "oneshot_1MiB": 256 << 10}
    for label, n in sizes.items():
        idx = torch.arange(n, dtype=torch.int32, device="cuda")
        base = ((idx * 11 + 5 * rank) % 1000).to(torch.float32)
        want0 = sum(((idx * 11 + 5 * r) % 1000).to(torch.float32) for r in range(world))
        y = torch.empty(n, dtype=torch.float32, device="cuda")
        wrong = 0
        for it in range(LL128_STRESS_CALLS):
            k = float(it % 113)
            xi = base + k
            c.all_reduce(xi.data_ptr(), y.data_ptr(), n, 7, 0, st)
            if not torch.equal(y, want0 + world * k):
                wrong += 1
        calls += LL128_STRESS_CALLS
        bad += wrong
        if wrong:
            res["ok"] = False
            res["errors"].append(f"ll128 forced stress {label} ({4 * n} B): {wrong} of {LL128_STRESS_CALLS} calls wrong")
    res["ll128_forced_checked_calls"] = calls
    res["ll128_forced_mismatched_calls"] = bad


# tests/test_multiprocess_gpu.py LL_CASES (kept equal by tests/test_tools_cpu.py):
# (kind, ncclDataType, op, count, byte offset of send / recv). GPUTEST_r05 saw
# this sequence, issued back to back on the default protocols, return wrong
# data from the Simple direct path at 8 ranks sharing one GPU (case 36); the
# node run replays it across the fabric.
MIXED_CASES = [
    ("ar", 7, 0, 1, 0), ("ar", 7, 0, 3, 0), ("ar", 7, 0, 1000, 0), ("ar", 7, 0, 16384, 0), ("ar", 6, 0, 17, 0),
    ("ar", 9, 4, 4097, 0), ("ar", 2, 4, 999, 0), ("ar", 4, 2, 4096, 0), ("ar", 10, 0, 33, 0),
    ("ar", 1, 3, 65536, 0), ("ar", 8, 1, 8191, 0), ("ar", 7, 0, 40000, 0), ("ar", 7, 0, 1001, 4),
    ("ar", 0, 0, 77, 3), ("rs", 7, 0, 1000, 0), ("rs", 6, 4, 333, 2), ("rs", 0, 2, 5, 1), ("rs", 4, 4, 4096, 0),
    ("rs", 7, 0, 20000, 0), ("red", 7, 0, 1000, 0), ("red", 9, 4, 777, 0), ("red", 2, 3, 64, 0),
    ("red", 7, 0, 123, 4), ("red", 7, 1, 4096, 0), ("ar", 7, 0, 64, 0),
    ("ar", 7, 0, 50003, 0), ("ar", 6, 4, 77777, 2), ("ar", 4, 2, 30000, 8), ("rs", 7, 0, 30001, 4),
    ("rs", 2, 2, 131072, 0), ("red", 7, 0, 99999, 0), ("red", 8, 4, 100000, 8),
    ("ar", 7, 4, 262144, 0), ("ar", 9, 0, 300001, 0), ("ar", 11, 0, 600001, 1), ("ar", 7, 0, 300000, 4),
    ("ar", 2, 2, 1000003, 0), ("ar", 8, 0, 200001, 0), ("red", 7, 0, 300001, 0), ("red", 9, 4, 200003, 2),
    ("red", 2, 3, 500000, 0),
    ("ar", 7, 0, 1100000, 0), ("rs", 7, 4, 1048577, 0),
]
MIXED_ITERS = 3
_EB = {0: 1, 1: 1, 2: 4, 3: 4, 4: 8, 5: 8, 6: 2, 7: 4, 8: 8, 9: 2, 10: 1, 11: 1}


def _mixed_op(op):
    """The leg's op for a case: max / min kept, everything else a sum of small
    integers (Prod -> max) — every fold order then gives the same bits, so a
    GPU restatement checks the output exactly; the kinds, types, sizes and
    offsets (hence protocols, grids and staging slices) are the case's own."""
    return op if op in (2, 3) else (2 if op == 1 else 0)


def _mixed_input(torch, dt, op, total, seed, device="cuda"):
    """Raw bytes of one rank's input: full-range values for max / min (finite
    floats, no zeros or NaN codes for fp8), small integers for sums."""
    g = torch.Generator(device=device).manual_seed(seed)
    if op == 0:
        v = torch.randint(0, 16 if dt not in (10, 11) else 2, (total,), generator=g, device=device)
        if dt in (10, 11):
            return v.to(torch.float32).to(torch.float8_e4m3fn if dt == 10 else torch.float8_e5m2).view(torch.uint8)
        tdt = {0: torch.int8, 1: torch.uint8, 2: torch.int32, 3: torch.int32, 4: torch.int64, 5: torch.int64,
               6: torch.float16, 7: torch.float32, 8: torch.float64, 9: torch.bfloat16}[dt]
        return v.to(tdt).view(torch.uint8)
    if dt in (6, 7, 8, 9):
        f = torch.randn(total, generator=g, device=device, dtype=torch.float64) * 1000
        return f.to({6: torch.float16, 7: torch.float32, 8: torch.float64, 9: torch.bfloat16}[dt]).view(torch.uint8)
    c = torch.randint(0, 256, (total * _EB[dt],), generator=g, device=device, dtype=torch.int64).to(torch.uint8)
    if dt == 10:
        c[((c & 0x7f) == 0x7f) | (c == 0x80)] = 0x01
    elif dt == 11:
        c[((c & 0x7c) == 0x7c) | (c == 0x80)] = 0x01
    return c


def _mixed_expected(torch, dt, op, ins):
    """The exact result of the leg's op over every rank's raw input bytes."""
    if op == 0:
        if dt in (10, 11):
            f8 = torch.float8_e4m3fn if dt == 10 else torch.float8_e5m2
            return sum(x.view(f8).float() for x in ins).to(f8).view(torch.uint8)
        if dt in (6, 7, 8, 9):
            tdt = {6: torch.float16, 7: torch.float32, 8: torch.float64, 9: torch.bfloat16}[dt]
            return sum(x.view(tdt).double() for x in ins).to(tdt).view(torch.uint8)
        tdt = {0: torch.int8, 1: torch.uint8, 2: torch.int32, 3: torch.int32, 4: torch.int64, 5: torch.int64}[dt]
        return sum(x.view(tdt).to(torch.int64) for x in ins).to(tdt).view(torch.uint8)
    pick = torch.maximum if op == 2 else torch.minimum
    if dt in (10, 11):
        f8 = torch.float8_e4m3fn if dt == 10 else torch.float8_e5m2
        acc = ins[0].view(f8).float()
        for x in ins[1:]:
            acc = pick(acc, x.view(f8).float())
        return acc.to(f8).view(torch.uint8)
    if dt in (6, 7, 8, 9):
        tdt = {6: torch.float16, 7: torch.float32, 8: torch.float64, 9: torch.bfloat16}[dt]
        acc = ins[0].view(tdt).double()
        for x in ins[1:]:
            acc = pick(acc, x.view(tdt).double())
        return acc.to(tdt).view(torch.uint8)
    tdt = {0: torch.int8, 1: torch.uint8, 2: torch.int32, 3: torch.int32, 4: torch.int64, 5: torch.int64}[dt]
    flip = {3: -(1 << 31), 5: -(1 << 63)}.get(dt)   # unsigned: compare with the sign bit flipped
    vs = [x.view(tdt) if flip is None else (x.view(tdt) ^ flip) for x in ins]
    acc = vs[0]
    for v in vs[1:]:
        acc = pick(acc, v)
    return (acc if flip is None else acc ^ flip).view(torch.uint8)


def mixed_sequence(comm, rank, world, st, res, iters=MIXED_ITERS):
    """MIXED_CASES back to back on the default protocols (no host sync between
    calls, inputs new every iteration, every rank's input regenerated on each
    rank from its seed), every output checked exactly on the GPU; per-rank
    counts of checked and wrong calls, and the first wrong call described."""
    import torch
    checked = bad = 0
    first = None
    for it in range(iters):
        keep = []
        for i, (kind, dt, op0, count, shift) in enumerate(MIXED_CASES):
            op = _mixed_op(op0)
            eb = _EB[dt]
            total = count * world if kind == "rs" else count
            x = _mixed_input(torch, dt, op, total, 50000 * it + 100 * i + rank)
            tx = torch.zeros(total * eb + 16, dtype=torch.uint8, device="cuda")
            tx[shift:shift + total * eb] = x
            out_b = count * eb
            ty = torch.full((out_b + 16,), 0xA5, dtype=torch.uint8, device="cuda")
            root = (i * 3 + 1) % world
            sp, rp = tx.data_ptr() + shift, ty.data_ptr() + shift
            if kind == "ar":
                comm.all_reduce(sp, rp, count, dt, op, st)
            elif kind == "rs":
                comm.reduce_scatter(sp, rp, count, dt, op, st)
            else:
                comm.reduce(sp, rp, count, dt, op, root, st)
            keep.append((i, kind, dt, op, count, shift, root, tx, ty))
        torch.cuda.synchronize()
        for i, kind, dt, op, count, shift, root, tx, ty in keep:
            if kind == "red" and rank != root:
                continue
            eb = _EB[dt]
            total = count * world if kind == "rs" else count
            ins = [_mixed_input(torch, dt, op, total, 50000 * it + 100 * i + r) for r in range(world)]
            want = _mixed_expected(torch, dt, op, ins)
            if kind == "rs":
                want = want[rank * count * eb:(rank + 1) * count * eb]
            got = ty[shift:shift + count * eb]
            checked += 1
            if not torch.equal(got, want):
                bad += 1
                if first is None:
                    w = (got.view(-1, eb) != want.view(-1, eb)).any(dim=1).nonzero().flatten()
                    first = (f"iteration {it} case {i} {MIXED_CASES[i]} (leg op {op}): {w.numel()} of {count} "
                             f"elements wrong, first {int(w[0])} last {int(w[-1])}")
        del keep
    res["mixed_seq_checked_calls"] = checked
    res["mixed_seq_mismatches"] = bad
    if bad:
        res["ok"] = False
        res["errors"].append(f"mixed sequence: {bad} of {checked} calls wrong; {first}")


LINK_PROBE_BYTES = 256 << 20   # per peer per launch


def link_probe(lib, comm, st, res):
    """The fabric's per-link rate (what config D is priced against, bench.py
    add_fabric_rates): every rank pushes to, then pulls from, every peer's
    staging at once (nbxDebugLinkProbe). The probe overwrites the peers'
    staging slices, so the communicator is kept quiet around it: a small
    AllReduce (LL, not the staging) after each rank's stream drained, before
    the first probe and after the last — no peer is still in a Simple call
    when the probes start, or still probing when the next one starts."""
    import ctypes
    import torch
    lib.nbxDebugLinkProbe.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.POINTER(ctypes.c_size_t)]
    moved = ctypes.c_size_t(0)

    def quiet():
        torch.cuda.synchronize()
        for f in _ALIGN:
            f()
        torch.cuda.synchronize()

    for pull, name in ((0, "push"), (1, "pull")):
        def probe():
            rc_ = lib.nbxDebugLinkProbe(comm.handle, LINK_PROBE_BYTES, pull, 0, st, ctypes.byref(moved))
            if rc_ != 0:
                raise RuntimeError(f"nbxDebugLinkProbe: {rc_}")
        quiet()
        res[f"link_{name}_ms"] = _time_calls(probe, ITERS)
    quiet()
    res["link_bytes_per_peer"] = int(moved.value)


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
    al_x = torch.ones(16, device="cuda")
    al_y = torch.empty_like(al_x)
    _ALIGN[:] = [lambda: comm.all_reduce(al_x.data_ptr(), al_y.data_ptr(), 16, F32, SUM, st)]

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

    # LL128 in the default protocol set (bit 1): off by default across GPUs
    # (comm_mp_init.cc protoGateAcrossGpus), and dropped by the creation-time probe
    # if it saw a torn line
    import ctypes
    lib = nbx.load_library()
    lib.nbxDebugCommProtoMask.argtypes = [ctypes.c_void_p]
    lib.nbxDebugCommProtoMask.restype = ctypes.c_int
    lib.nbxDebugCommSettings.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
    lib.nbxDebugTransportAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                               ctypes.c_void_p, ctypes.c_void_p]
    res["proto_mask"] = int(lib.nbxDebugCommProtoMask(comm.handle))
    res["ll128_active"] = bool(res["proto_mask"] & 2)
    res["ipc_repairs"] = {"direct": _ipc_repairs(lib, comm), "ring": _ipc_repairs(lib, comm_ring)}
    _progress("communicators ready", res)
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
    # the xGMI transport alone — the direct AllReduce schedule's
    # pushes and gather of the same 1 GiB with the fold reduced to a copy
    # (nbxDebugTransportAllReduce); its output is junk, y is rewritten below
    def xport():
        rc_ = lib.nbxDebugTransportAllReduce(x.data_ptr(), y.data_ptr(), COUNT, F32, comm.handle, st)
        if rc_ != 0:
            raise RuntimeError(f"nbxDebugTransportAllReduce: {rc_}")
    xport()
    torch.cuda.synchronize()
    res["transport_allreduce_ms"] = _time_calls(xport, ITERS)
    link_probe(lib, comm, st, res)
    _progress("config D timed", res)
    simple_knob_sweep(ids[6:6 + len(SIMPLE_KNOBS)], rank, world, st, x, y, exp, res)
    _progress("Simple knobs timed", res)
    # the large-message curve between the sweep (<= 16 MiB) and config D
    # (1 GiB) on the default communicator, each size checked once
    curve = []
    for b in CURVE_BYTES:
        n = b // 4
        y.zero_()
        comm.all_reduce(x.data_ptr(), y.data_ptr(), n, F32, SUM, st)
        torch.cuda.synchronize()
        check(f"allreduce_{b >> 20}MiB", y[:n], exp[:n])
        curve.append(_time_calls(lambda: comm.all_reduce(x.data_ptr(), y.data_ptr(), n, F32, SUM, st), ITERS))
    res["curve_bytes"] = list(CURVE_BYTES)
    res["curve_allreduce_ms"] = curve

    # Simple path with inputs that change every call (direct and ring schedules,
    # 32 MiB): catches any stale peer data a cache could serve across calls
    xs_ = x[:SIMPLE_STRESS_COUNT]
    es_ = exp[:SIMPLE_STRESS_COUNT]
    ys_ = torch.empty(SIMPLE_STRESS_COUNT, dtype=torch.float32, device="cuda")
    for name, c in (("direct", comm), ("ring", comm_ring)):
        bad = 0
        for it in range(SIMPLE_STRESS_ITERS):
            xi = xs_ + float(it % 89)
            c.all_reduce(xi.data_ptr(), ys_.data_ptr(), SIMPLE_STRESS_COUNT, F32, SUM, st)
            if not torch.equal(ys_, es_ + float(world * (it % 89))):
                bad += 1
        if bad:
            res["ok"] = False
            res["errors"].append(f"simple_{name}_stress: {bad} of {SIMPLE_STRESS_ITERS} calls wrong")
    res["simple_stress_checked_calls"] = 2 * SIMPLE_STRESS_ITERS
    del xs_, es_, ys_
    _progress("config D done", res)
    mixed_sequence(comm, rank, world, st, res)
    _progress("mixed sequence done", res)
    # 1 MiB on the default protocol set (LL128 on one GPU; across GPUs LL128
    # is off by default, so Simple carries it there): exact on every one of
    # LL128_ITERS calls with inputs that change per call (a torn line or a
    # stale slot would show up as a wrong value), then the per-call latency
    # (LL128 forced across GPUs: ll128_stress in the protocol sweep)
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

    del x, y, yr, exp, x1, e1, y1, xs, ys
    torch.cuda.empty_cache()
    _progress("LL / LL128 done", res)
    config_e(comm, rank, world, st, res)
    _progress("config E done", res)
    protocol_sweep(ids[2:6], rank, world, st, "NBX_BENCH_DEVICE" in os.environ, res)
    _progress("protocol sweep done", res)

    torch.cuda.synchronize()
    if comm.async_error() != 0 or comm_ring.async_error() != 0:
        res["ok"] = False
        res["errors"].append("async error")
    comm_ring.destroy()
    comm.destroy()
    return res


def _blocks(count, eb, n):
    """The direct schedule's AllReduce blocks (nccl_api.cc blockRange): 16-byte aligned."""
    epp = 16 // eb
    per = -(-count // n)
    per = -(-per // epp) * epp
    return [(min(count, per * b), min(count, per * b + per)) for b in range(n)]


def config_e(comm, rank, world, st, res):
    """SURVEY §8(d) config E across the N GPUs: ncclAllReduce int64 ncclMax over
    128 MiB (full-range random bits) and fp8 e4m3 ncclSum over 128 MiB (random
    finite codes), checked bit-exact against a GPU restatement on the same
    seeded inputs (every rank regenerates every rank's input): max is
    order-free; the fp8 sum folds each block c in the direct schedule's order
    c+1, ..., c with an fp32 add and a saturating RNE narrowing per step
    (SATFINITE: clamp to +-448, then torch's cast; NaN = any NaN code)."""
    import torch
    I64, F8, MAX, SUM = 4, 10, 2, 0

    def gen_i64(r):
        g = torch.Generator(device="cuda").manual_seed(9001 + r)
        return torch.randint(-2**63, 2**63 - 1, (E_I64,), dtype=torch.int64, device="cuda", generator=g)

    def gen_f8(r):
        g = torch.Generator(device="cuda").manual_seed(7001 + r)
        c = torch.randint(0, 256, (E_F8,), dtype=torch.uint8, device="cuda", generator=g)
        c[(c & 0x7f) == 0x7f] = 0   # finite codes only
        return c

    # int64 max
    x = gen_i64(rank)
    y = torch.empty_like(x)
    comm.all_reduce(x.data_ptr(), y.data_ptr(), E_I64, I64, MAX, st)
    torch.cuda.synchronize()
    exp = gen_i64(0)
    for r in range(1, world):
        exp = torch.maximum(exp, gen_i64(r))
    ok_i = torch.equal(y, exp)
    res["config_e_int64_max_ms"] = _time_calls(lambda: comm.all_reduce(x.data_ptr(), y.data_ptr(), E_I64, I64, MAX,
                                                                       st), ITERS)
    del x, y, exp
    # fp8 e4m3 sum
    xs = [gen_f8(r) for r in range(world)]
    y = torch.empty(E_F8, dtype=torch.uint8, device="cuda")
    comm.all_reduce(xs[rank].data_ptr(), y.data_ptr(), E_F8, F8, SUM, st)
    torch.cuda.synchronize()
    f8 = torch.float8_e4m3fn
    exp = torch.empty(E_F8, dtype=torch.uint8, device="cuda")
    for c, (lo, hi) in enumerate(_blocks(E_F8, 1, world)):
        if hi <= lo:
            continue
        acc = xs[(c + 1) % world][lo:hi].view(f8)
        for q in range(1, world):
            acc = (acc.float() + xs[(c + 1 + q) % world][lo:hi].view(f8).float()).clamp(-448.0, 448.0).to(f8)
        exp[lo:hi] = acc.view(torch.uint8)
    nan_e = (exp & 0x7f) == 0x7f
    nan_g = (y & 0x7f) == 0x7f
    ok_f = bool(((y == exp) | (nan_e & nan_g)).all().item())
    res["config_e_fp8_nan_fraction"] = round(float(nan_e.float().mean().item()), 4)
    res["config_e_fp8_saturated_fraction"] = round(float(((exp & 0x7f) == 0x7e).float().mean().item()), 4)
    res["config_e_fp8_sum_ms"] = _time_calls(lambda: comm.all_reduce(xs[rank].data_ptr(), y.data_ptr(), E_F8, F8, SUM,
                                                                      st), ITERS)
    del xs, y, exp
    torch.cuda.empty_cache()
    for name, ok in (("config_e_int64_max", ok_i), ("config_e_fp8_sum", ok_f)):
        if not ok:
            res["ok"] = False
            res["errors"].append(f"{name}: output differs from the bit-exact restatement")


# direct, ring, the protocol sweep's four, the Simple knobs'
N_IDS = 6 + len(SIMPLE_KNOBS)


def main():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dev = int(os.environ.get("NBX_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    os.environ.setdefault("NBX_TIMEOUT_SEC", "60")
    os.environ.setdefault("NBX_BOOTSTRAP_TIMEOUT", "120")
    # (rehearsals with every rank on one GPU need no grid caps: the communicator
    # splits the GPU's CUs among the ranks that share it, for every protocol)
    for line in sys.stdin:
        parts = line.split()
        if not parts:
            continue
        if parts[0] == "ID":
            nbx = _pkg()   # imports torch first (one HIP runtime); no GPU use: the root is a host thread
            _emit("ID " + " ".join(bytes(nbx.get_unique_id()).hex() for _ in range(N_IDS)))
        elif parts[0] == "RUN":
            try:
                res = run(parts[1:1 + N_IDS], rank, world, dev)
            except Exception as e:   # reported to the parent, never raised past it
                res = {"rank": rank, "ok": False, "errors": [f"{type(e).__name__}: {e}"]}
            _emit("RESULT " + json.dumps(res))
            return 0
        elif parts[0] == "QUIT":
            return 0
    return 0


if __name__ == "__main__":
    sys.exit(main())
