#!/usr/bin/env python3
"""probe_ipc_reuse.py — root-cause probe for the round-2 N=2 Simple-path
wrong result: does a hipIpc import of a peer's NEW
allocation ever show another allocation's bytes, and if so, is it (a) an IPC
handle whose bytes repeat an earlier handle of a different allocation (a cache
keyed by handle bytes then serves the old mapping), or (b) a fresh import that
lands on a virtual address this process freed or unmapped before (a stale
translation)?

Two processes on GPU 0, raw HIP through ctypes (no torch, no libnbxccl
control plane). Rank 0 allocates a buffer per iteration (sizes 2 MiB..256
MiB), fills it with a per-iteration word, exports its handle. Rank 1 churns
its own allocations (hipMalloc/hipFree of random sizes, like the caching
allocator's empty_cache), maps the handle according to the mode, reads the
first and last 4 KiB through the mapping (hipMemcpy DtoH: a copy kernel),
writes a per-iteration word through it (hipMemsetD32: a fill kernel), and
rank 0 checks that the write landed. Modes:
  close   — open, use, close (per-call import, no cache)
  cache   — mapPeer's cache: a mapping keyed by the 64 handle bytes is reused
  retire  — open, use, never close (round 2's retired list)
Prints one JSON line per mode: failures and, per failure, whether the handle
bytes had been seen before and whether the mapped address was one this rank
had freed (own allocation) or closed (import) earlier.
"""
from __future__ import annotations

import ctypes
import json
import multiprocessing as mp
import os
import random
import sys

SIZES = [2 << 20, 4 << 20, 20 << 20, 64 << 20, 256 << 20]
OWN_SIZES = [2 << 20, 20 << 20, 128 << 20, 512 << 20]


class _Handle(ctypes.Structure):   # hipIpcMemHandle_t, passed BY VALUE
    _fields_ = [("reserved", ctypes.c_char * 64)]


def _hip():
    lib = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.hipSetDevice.argtypes = [ctypes.c_int]
    lib.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
    lib.hipFree.argtypes = [vp]
    lib.hipMemsetD32.argtypes = [vp, ctypes.c_int, sz]
    lib.hipMemcpy.argtypes = [vp, vp, sz, ctypes.c_int]
    lib.hipDeviceSynchronize.argtypes = []
    lib.hipIpcGetMemHandle.argtypes = [ctypes.c_char_p, vp]
    lib.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(vp), _Handle, ctypes.c_uint]
    lib.hipIpcCloseMemHandle.argtypes = [vp]
    lib.hipMemGetAddressRange.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(sz), vp]
    return lib


def _ck(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {rc}")


def _malloc(h, n):
    p = ctypes.c_void_p()
    _ck(h.hipMalloc(ctypes.byref(p), n), "hipMalloc")
    return p.value


def _words(h, p, n_bytes):
    buf = (ctypes.c_uint32 * (n_bytes // 4))()
    _ck(h.hipMemcpy(ctypes.cast(buf, ctypes.c_void_p), ctypes.c_void_p(p), n_bytes, 2), "hipMemcpy DtoH")
    return list(buf)


def rank0(conn, iters, seed):
    h = _hip()
    _ck(h.hipSetDevice(0), "hipSetDevice")
    rng = random.Random(seed)
    live = []
    exported = {}   # address -> iteration of its last export
    for i in range(iters):
        size = rng.choice(SIZES)
        p = _malloc(h, size)
        _ck(h.hipMemsetD32(ctypes.c_void_p(p), 0x10000000 + i, size // 4), "memset")
        _ck(h.hipDeviceSynchronize(), "sync")
        hb = ctypes.create_string_buffer(64)
        rc = h.hipIpcGetMemHandle(hb, ctypes.c_void_p(p))
        if rc != 0:   # record and go on: the address / earlier export pattern is the clue
            conn.send(("export_failed", i, rc, size, p, exported.get(p)))
            conn.recv()
            _ck(h.hipFree(ctypes.c_void_p(p)), "hipFree")
            continue
        exported[p] = i
        conn.send(("buf", i, hb.raw, size, p))
        conn.recv()   # rank 1 has read and written through its mapping
        head = _words(h, p, 4096)
        tail = _words(h, p + size - 4096, 4096)
        want = 0x20000000 + i
        conn.send(all(w == want for w in head) and all(w == want for w in tail))
        if rng.random() < 0.8:
            _ck(h.hipFree(ctypes.c_void_p(p)), "hipFree")
        else:
            live.append(p)
            if len(live) > 4:
                _ck(h.hipFree(ctypes.c_void_p(live.pop(0))), "hipFree")
    conn.send(("end",))
    conn.recv()


def rank1(conn, mode, seed, out_q):
    try:
        _rank1(conn, mode, seed, out_q)
    except Exception as e:   # report, never strand the parent
        out_q.put({"mode": mode, "error": f"{type(e).__name__}: {e}"})


def _rank1(conn, mode, seed, out_q):
    h = _hip()
    _ck(h.hipSetDevice(0), "hipSetDevice")
    rng = random.Random(seed + 1)
    own = []
    freed_own = set()     # base addresses this process hipFree'd
    closed_maps = set()   # addresses of imports this process closed
    seen_handles = {}     # handle bytes -> iteration first seen
    cache = {}            # mode "cache": handle bytes -> mapped address
    fails, n = [], 0
    export_fails = []
    while True:
        msg = conn.recv()
        if msg[0] == "end":
            conn.send(None)
            break
        if msg[0] == "export_failed":
            _, i, rc, size, paddr, prev = msg
            export_fails.append({"iter": i, "rc": rc, "size": size, "addr": hex(paddr),
                                 "same_addr_exported_at_iter": prev})
            conn.send(None)
            continue
        _, i, hraw, size, peer_addr = msg
        # own allocation churn (the caching allocator's malloc / empty_cache)
        for _ in range(rng.randint(0, 3)):
            if own and rng.random() < 0.6:
                p = own.pop(rng.randrange(len(own)))
                _ck(h.hipFree(ctypes.c_void_p(p)), "hipFree own")
                freed_own.add(p)
            else:
                own.append(_malloc(h, rng.choice(OWN_SIZES)))
        handle_seen = seen_handles.get(hraw)
        seen_handles.setdefault(hraw, i)
        hit = mode == "cache" and hraw in cache
        if hit:
            va = cache[hraw]
        else:
            pv = ctypes.c_void_p()
            _ck(h.hipIpcOpenMemHandle(ctypes.byref(pv), _Handle.from_buffer_copy(hraw), 1),
                "hipIpcOpenMemHandle")
            va = pv.value
        reused_from = ("own_freed" if va in freed_own else "closed_import" if va in closed_maps else None)
        want = 0x10000000 + i
        head = _words(h, va, 4096)
        tail = _words(h, va + size - 4096, 4096)
        read_ok = all(w == want for w in head) and all(w == want for w in tail)
        _ck(h.hipMemsetD32(ctypes.c_void_p(va), 0x20000000 + i, 1024), "memset head")
        _ck(h.hipMemsetD32(ctypes.c_void_p(va + size - 4096), 0x20000000 + i, 1024), "memset tail")
        _ck(h.hipDeviceSynchronize(), "sync")
        conn.send(None)
        write_ok = conn.recv()
        n += 1
        if not (read_ok and write_ok):
            fails.append({"iter": i, "size": size, "read_ok": read_ok, "write_ok": write_ok,
                          "cache_hit": hit, "handle_seen_at_iter": handle_seen, "va_reused_from": reused_from,
                          "read_head_word": hex(head[0]), "want": hex(want)})
        if mode == "close":
            _ck(h.hipIpcCloseMemHandle(ctypes.c_void_p(va)), "close")
            closed_maps.add(va)
        elif mode == "cache":
            cache[hraw] = va
    out_q.put({"mode": mode, "iters": n, "failures": len(fails), "distinct_handles": len(seen_handles),
               "first_failures": fails[:8], "export_failures": len(export_fails),
               "first_export_failures": export_fails[:8]})


def run_mode(mode, iters, seed):
    ctx = mp.get_context("spawn")
    a, b = ctx.Pipe()
    q = ctx.Queue()
    p0 = ctx.Process(target=rank0, args=(a, iters, seed), daemon=True)
    p1 = ctx.Process(target=rank1, args=(b, mode, seed, q), daemon=True)
    p0.start()
    p1.start()
    res = q.get(timeout=100)
    p1.join(30)
    for p in (p0, p1):
        if p.is_alive():
            p.terminate()
    return res


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 150
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["close", "cache", "retire"]
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for m in modes:
        print(json.dumps(run_mode(m, iters, 1234)), flush=True)


if __name__ == "__main__":
    main()
