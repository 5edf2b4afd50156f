#!/usr/bin/env python3
"""probe_ipc_export.py — why did hipIpcGetMemHandle refuse a fresh connection
buffer (gpurun_out/r3s/test_mp.log:43: the second
ncclCommSplit child of a 4-rank test, rank 2, 'invalid argument' on the LL
buffer of a 3-rank communicator)?

Raw HIP through ctypes, no libnbxccl. N processes on GPU 0 replay the
library's communicator lifecycle (comm_mp_init.cc mpInit / mpFreeState) cycle
after cycle: each rank allocates the four connection buffers a communicator
of n ranks allocates (LL lines, LL128 lines, Simple staging, Simple flag
words — the library's own sizes for that n and grid), takes an IPC handle of
each at once, the handles are all-gathered, every rank opens every peer's
handles, writes a word through each mapping and checks its own buffers, then
the communicator is torn down (imports closed, buffers freed). Like
ncclCommSplit, a cycle sometimes keeps the previous generation alive while
the next one is created, and between cycles each rank churns ordinary
allocations (the caching allocator's malloc / empty_cache). Modes:
  uc-raw   hipExtMallocWithFlags(hipDeviceMallocUncached), the exact size
           (the library until round 3's fix)
  uc-2m    the same, size rounded up to whole 2 MiB pages (the library now)
  cg-raw   plain hipMalloc, exact size
  cg-2m    plain hipMalloc, 2 MiB pages
A "-pool" part keeps every exported buffer for the life of the process: a
torn-down generation's buffers go to a pool keyed by size and the next
allocation of that size reuses one (re-exported, re-imported by the peers).
A "-bar" suffix tears a generation down in two steps: every rank closes its
imports, all ranks meet, then the owners free; without it a rank frees its
own buffers right after closing its imports, while peers may still have them
mapped (the library's ncclCommDestroy: no barrier).
For every refused export it records the size, the pointer's offset inside a
2 MiB page, and hipMemGetAddressRange's base / size for the pointer (is the
buffer its own allocation, or a piece of a larger one?). One JSON line per
mode.
"""
from __future__ import annotations

import ctypes
import json
import multiprocessing as mp
import os
import random
import sys

PAGE = 2 << 20
UNCACHED = 0x3   # hipDeviceMallocUncached


class _Handle(ctypes.Structure):   # hipIpcMemHandle_t, passed BY VALUE
    _fields_ = [("reserved", ctypes.c_char * 64)]


def _hip():
    lib = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.hipSetDevice.argtypes = [ctypes.c_int]
    lib.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
    lib.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
    lib.hipFree.argtypes = [vp]
    lib.hipMemsetD32.argtypes = [vp, ctypes.c_int, sz]
    lib.hipMemcpy.argtypes = [vp, vp, sz, ctypes.c_int]
    lib.hipDeviceSynchronize.argtypes = []
    lib.hipGetLastError.argtypes = []
    lib.hipIpcGetMemHandle.argtypes = [ctypes.c_char_p, vp]
    lib.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(vp), _Handle, ctypes.c_uint]
    lib.hipIpcCloseMemHandle.argtypes = [vp]
    lib.hipMemGetAddressRange.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(sz), vp]
    return lib


def _ck(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {rc}")


def conn_sizes(n, grid):
    """The four connection buffers of an n-rank communicator (comm_mp_init.cc mpAllocLL / mpInit defaults)."""
    ll_slot = 2 * ((64 << 10) // 8)
    ll = (2 * n * ll_slot + n + 1) * 8
    half = (4 << 20) // 2
    l128_slot = 2 * ((half + 47) // 48)
    l128 = 2 * n * l128_slot * 64 if n <= 8 else 0
    cells = n * grid
    stage = 2 * 2 * cells * (64 << 10)
    sflags = 4 * cells * 8
    return [("ll", ll), ("l128", l128), ("stage", stage), ("sflags", sflags)]


def rank_main(rank, conn, mode, cycles, seed, q):
    try:
        q.put(_rank(rank, conn, mode, cycles, seed))
    except Exception as e:   # report, never strand the parent
        q.put({"rank": rank, "error": f"{type(e).__name__}: {e}"})
        try:
            conn.send(("dead",))
        except Exception:
            pass


def _rank(rank, conn, mode, cycles, seed):
    h = _hip()
    _ck(h.hipSetDevice(0), "hipSetDevice")
    rng = random.Random(seed * 131 + rank)
    uncached = mode.startswith("uc")
    rounded = "-2m" in mode
    barrier = "-bar" in mode
    pooled = "-pool" in mode   # exported buffers are never freed: a size-keyed pool reuses them
    pool, pool_hits = {}, 0

    def release(b):
        if pooled:
            pool.setdefault(b[1], []).append(b[0])
        else:
            _ck(h.hipFree(ctypes.c_void_p(b[0])), "hipFree")
            freed.add(b[0])
    own = []                 # ordinary allocations (churn)
    gens = []                # live communicator generations: (own bufs, imports)
    freed, closed, exported = set(), set(), set()
    retry_ok = retry_fail = new_alloc_ok = new_alloc_fail = 0
    exports = fails = bad_reads = 0
    fail_detail, bad_detail, canary_detail = [], [], []
    canary_bad = canary_err = 0
    seen_handles, va_handle, handle_samples = {}, {}, []
    canary_err_detail = []
    sub_alloc = 0            # buffers whose pointer is not its allocation's base
    size_mismatch = 0        # buffers whose allocation range differs from the requested bytes
    for cyc in range(cycles):
        n, grid = conn.recv()
        exported_prev = set(exported)   # addresses exported (then freed) in earlier cycles
        # allocation churn of this rank's ordinary memory
        for _ in range(rng.randint(0, 4)):
            if own and rng.random() < 0.5:
                p = own.pop(rng.randrange(len(own)))
                _ck(h.hipFree(ctypes.c_void_p(p)), "hipFree own")
                freed.add(p)
            else:
                p = ctypes.c_void_p()
                _ck(h.hipMalloc(ctypes.byref(p), rng.choice([4096, 1 << 20, 3 << 20, 64 << 20])), "hipMalloc own")
                own.append(p.value)
        bufs, handles, info = [], [], []
        for name, size in conn_sizes(n, grid):
            if size == 0:
                handles.append(None)
                bufs.append(None)
                continue
            bytes_ = (size + PAGE - 1) // PAGE * PAGE if rounded else size
            p = ctypes.c_void_p()
            if pooled and pool.get(bytes_):
                p.value = pool[bytes_].pop()   # an exported buffer of this size, never freed: reused
                pool_hits += 1
            elif uncached:
                _ck(h.hipExtMallocWithFlags(ctypes.byref(p), bytes_, UNCACHED), "hipExtMallocWithFlags")
            else:
                _ck(h.hipMalloc(ctypes.byref(p), bytes_), "hipMalloc")
            base, rsz = ctypes.c_void_p(), ctypes.c_size_t()
            _ck(h.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(rsz), p), "hipMemGetAddressRange")
            if base.value != p.value:
                sub_alloc += 1
            if rsz.value != bytes_:
                size_mismatch += 1
            _ck(h.hipMemsetD32(p, 0, min(1024, bytes_ // 4)), "memset")
            # canary in the last 16 bytes: what an importer must read through its mapping
            _ck(h.hipMemsetD32(ctypes.c_void_p(p.value + bytes_ - 16), 0x70000000 + cyc * 8 + rank, 4), "canary")
            hb = ctypes.create_string_buffer(64)
            rc = h.hipIpcGetMemHandle(hb, p)
            exports += 1
            if rc != 0:
                h.hipGetLastError()
                fails += 1
                # the same pointer again: a deterministic refusal of this allocation?
                rc2 = h.hipIpcGetMemHandle(hb, p)
                h.hipGetLastError()
                if rc2 == 0:
                    retry_ok += 1
                else:
                    retry_fail += 1
                    # a fresh allocation (the refused one kept, so the address differs)
                    q2 = ctypes.c_void_p()
                    if uncached:
                        _ck(h.hipExtMallocWithFlags(ctypes.byref(q2), bytes_, UNCACHED), "hipExtMallocWithFlags")
                    else:
                        _ck(h.hipMalloc(ctypes.byref(q2), bytes_), "hipMalloc")
                    rc3 = h.hipIpcGetMemHandle(hb, q2)
                    h.hipGetLastError()
                    new_alloc_ok += rc3 == 0
                    new_alloc_fail += rc3 != 0
                    _ck(h.hipFree(q2), "hipFree")
                if len(fail_detail) < 12:
                    fail_detail.append({"cycle": cyc, "n": n, "buf": name, "bytes": bytes_, "rc": rc, "retry_rc": rc2,
                                        "offset_in_2MiB": p.value % PAGE, "base_is_ptr": base.value == p.value,
                                        "range_bytes": rsz.value, "addr_freed_before": p.value in freed,
                                        "addr_exported_before": p.value in exported,
                                        "addr_was_import": p.value in closed})
                handles.append(hb.raw if rc2 == 0 else None)
                if rc2 == 0:
                    exported.add(p.value)
            else:
                handles.append(hb.raw)
                exported.add(p.value)
            bufs.append((p.value, bytes_))
        _ck(h.hipDeviceSynchronize(), "sync")
        conn.send(("handles", handles))
        peers = conn.recv()          # every rank's handles
        imports = []
        sizes_k = [((sz + PAGE - 1) // PAGE * PAGE if rounded else sz) for _, sz in conn_sizes(n, grid)]
        for j, hs in enumerate(peers):
            if j == rank:
                continue
            for k, hraw in enumerate(hs):
                if hraw is None:
                    continue
                va = ctypes.c_void_p()
                _ck(h.hipIpcOpenMemHandle(ctypes.byref(va), _Handle.from_buffer_copy(hraw), 1), "hipIpcOpenMemHandle")
                size_k = sizes_k[k]
                seen_before = seen_handles.get(hraw)
                seen_handles.setdefault(hraw, (j, cyc, k))
                va_prev_handle = va_handle.get(va.value)
                va_handle[va.value] = hraw
                if len(handle_samples) < 6 and cyc < 2:
                    handle_samples.append({"owner": j, "cycle": cyc, "buf": k, "hex": hraw.hex()})
                can = (ctypes.c_uint32 * 4)()
                rc = h.hipMemcpy(ctypes.cast(can, ctypes.c_void_p), ctypes.c_void_p(va.value + size_k - 16), 16, 2)
                if rc != 0:   # the runtime refuses a read of the mapping's last bytes: record, read no canary
                    h.hipGetLastError()
                    canary_err += 1
                    if len(canary_err_detail) < 4:
                        rng_b, rng_s = ctypes.c_void_p(), ctypes.c_size_t()
                        rr = h.hipMemGetAddressRange(ctypes.byref(rng_b), ctypes.byref(rng_s), va)
                        h.hipGetLastError()
                        canary_err_detail.append({"cycle": cyc, "owner": j, "buf": conn_sizes(n, grid)[k][0],
                                                  "bytes": size_k, "rc": rc, "range_rc": rr,
                                                  "mapped_range_bytes": rng_s.value,
                                                  "range_base_is_va": rng_b.value == va.value})
                elif any(w != 0x70000000 + cyc * 8 + j for w in can):
                    canary_bad += 1
                    if len(canary_detail) < 8:
                        canary_detail.append({"cycle": cyc, "owner": j, "buf": conn_sizes(n, grid)[k][0],
                                              "got": hex(can[0]), "want": hex(0x70000000 + cyc * 8 + j),
                                              "va_was_import": va.value in closed, "va_freed_own": va.value in freed,
                                              "handle_seen_before": seen_before,
                                              "va_last_import_same_handle": va_prev_handle == hraw if va_prev_handle
                                              else None})
                # rank's word in the peer's buffer: 16 bytes per writer at the start
                _ck(h.hipMemsetD32(ctypes.c_void_p(va.value + 16 * rank), 0x5000 + cyc * 64 + rank, 4), "memset peer")
                imports.append(va.value)
        _ck(h.hipDeviceSynchronize(), "sync")
        conn.send(("mapped",))
        conn.recv()                  # every rank wrote into every mapping
        for j, hs in enumerate(peers):
            if j == rank:
                continue
            for k, hraw in enumerate(hs):
                if hraw is None or handles[k] is None:
                    continue
                got = (ctypes.c_uint32 * 4)()
                _ck(h.hipMemcpy(ctypes.cast(got, ctypes.c_void_p), ctypes.c_void_p(bufs[k][0] + 16 * j), 16, 2),
                    "hipMemcpy")
                if any(w != 0x5000 + cyc * 64 + j for w in got):
                    bad_reads += 1
                    import time
                    time.sleep(0.1)
                    _ck(h.hipDeviceSynchronize(), "sync")
                    late = (ctypes.c_uint32 * 4)()
                    _ck(h.hipMemcpy(ctypes.cast(late, ctypes.c_void_p), ctypes.c_void_p(bufs[k][0] + 16 * j), 16, 2),
                        "hipMemcpy")
                    late_ok = all(w == 0x5000 + cyc * 64 + j for w in late)
                    if len(bad_detail) < 12:
                        bad_detail.append({"cycle": cyc, "buf": conn_sizes(n, grid)[k][0], "bytes": bufs[k][1],
                                           "writer": j, "got": [hex(w) for w in got],
                                           "want": hex(0x5000 + cyc * 64 + j),
                                           "owner_offset_in_2MiB": bufs[k][0] % PAGE,
                                           "owner_offset_in_4KiB": bufs[k][0] % 4096,
                                           "seen_100ms_later": late_ok, "addr_exported_before": bufs[k][0] in exported_prev})
        conn.send(("checked",))
        gens.append((bufs, imports))
        keep, = conn.recv()          # every rank checked; ncclCommSplit: the parent outlives the child's creation
        dying = gens[:len(gens) - keep]
        del gens[:len(gens) - keep]
        for gb, gi in dying:
            for va in gi:
                _ck(h.hipIpcCloseMemHandle(ctypes.c_void_p(va)), "close")
                closed.add(va)
            if not barrier:
                for b in gb:
                    if b is not None:
                        release(b)
        conn.send(("closed",))
        conn.recv()
        if barrier:
            for gb, gi in dying:
                for b in gb:
                    if b is not None:
                        release(b)
        conn.send(("freed",))
        conn.recv()
    conn.send(("end",))
    return {"rank": rank, "exports": exports, "export_failures": fails, "sub_allocated": sub_alloc,
            "same_ptr_retry_ok": retry_ok, "same_ptr_retry_refused": retry_fail,
            "new_alloc_ok": new_alloc_ok, "new_alloc_refused": new_alloc_fail,
            "range_size_differs": size_mismatch,
            "bad_reads": bad_reads, "failures": fail_detail, "bad_read_detail": bad_detail,
            "canary_bad": canary_bad, "canary_detail": canary_detail, "canary_read_refused": canary_err,
            "canary_read_refused_detail": canary_err_detail, "distinct_handles": len(seen_handles),
            "pool_hits": pool_hits,
            "handle_samples": handle_samples}


def run_mode(mode, nproc, cycles, seed):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pipes = [ctx.Pipe() for _ in range(nproc)]
    procs = [ctx.Process(target=rank_main, args=(r, pipes[r][1], mode, cycles, seed, q), daemon=True)
             for r in range(nproc)]
    for p in procs:
        p.start()
    conns = [a for a, _ in pipes]
    rng = random.Random(seed)
    dead = False
    try:
        for cyc in range(cycles):
            n = nproc   # every rank takes part; the grid follows the ranks sharing the GPU, as mpInit
            grid = min(128, 256 // n)
            if rng.random() < 0.3:
                grid = rng.choice([1, 7, 64, 85, 128])
            for c in conns:
                c.send((n, grid))
            msgs = [c.recv() for c in conns]
            if any(m[0] == "dead" for m in msgs):
                dead = True
                break
            allh = [m[1] for m in msgs]
            for c in conns:
                c.send(allh)
            keep = 1 if rng.random() < 0.4 else 0
            for step in ("mapped", "checked", "closed", "freed"):
                msgs = [c.recv() for c in conns]
                if any(m[0] == "dead" for m in msgs):
                    dead = True
                    break
                for c in conns:
                    c.send((keep,) if step == "checked" else None)
            if dead:
                break
        if not dead:
            for c in conns:
                c.recv()
        res = []
        for _ in range(nproc):
            try:
                res.append(q.get(timeout=20 if dead else 60))
            except Exception:
                break
    finally:
        for p in procs:
            p.join(10)
            if p.is_alive():
                p.terminate()
    agg = {"mode": mode, "ranks": nproc, "cycles": cycles}
    agg["exports"] = sum(r.get("exports", 0) for r in res)
    agg["export_failures"] = sum(r.get("export_failures", 0) for r in res)
    agg["sub_allocated"] = sum(r.get("sub_allocated", 0) for r in res)
    agg["range_size_differs"] = sum(r.get("range_size_differs", 0) for r in res)
    for k in ("same_ptr_retry_ok", "same_ptr_retry_refused", "new_alloc_ok", "new_alloc_refused"):
        agg[k] = sum(r.get(k, 0) for r in res)
    agg["bad_reads"] = sum(r.get("bad_reads", 0) for r in res)
    agg["errors"] = [r["error"] for r in res if "error" in r]
    agg["failures"] = [dict(f, rank=r["rank"]) for r in res for f in r.get("failures", [])][:12]
    agg["bad_read_detail"] = [dict(f, rank=r["rank"]) for r in res for f in r.get("bad_read_detail", [])][:12]
    agg["canary_bad"] = sum(r.get("canary_bad", 0) for r in res)
    agg["canary_read_refused"] = sum(r.get("canary_read_refused", 0) for r in res)
    agg["distinct_handles_per_rank"] = [r.get("distinct_handles") for r in res]
    agg["pool_hits"] = sum(r.get("pool_hits", 0) for r in res)
    agg["handle_samples"] = [h for r in res for h in r.get("handle_samples", [])][:6]
    agg["canary_read_refused_detail"] = [dict(f, rank=r["rank"]) for r in res
                                         for f in r.get("canary_read_refused_detail", [])][:6]
    agg["canary_detail"] = [dict(f, rank=r["rank"]) for r in res for f in r.get("canary_detail", [])][:8]
    return agg


def main():
    cycles = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["uc-raw", "uc-2m", "cg-raw", "cg-2m"]
    nproc = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for m in modes:
        print(json.dumps(run_mode(m, nproc, cycles, 4321)), flush=True)


if __name__ == "__main__":
    main()
