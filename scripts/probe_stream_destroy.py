#!/usr/bin/env python3
"""probe_stream_destroy.py — under the HIP runtime torch loads (the one the
library runs on in every torch process): does hipStreamDestroy return while the
stream's kernels still run, and does the next hipStreamCreate hand out the
destroyed stream's handle? (per-stream dynamic-tile counters.)
Queues ~20 ms of nbxReduceMulti launches on a raw stream, destroys it, and
times destroy and the remaining work; then 32 create / launch / destroy
cycles count handle reuse. Prints one JSON line."""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    nbx.load_library()
    torch.cuda.set_device(0)
    hip = ctypes.CDLL("libamdhip64.so.7")   # already loaded by torch: the same runtime
    vp = ctypes.c_void_p
    hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
    hip.hipStreamDestroy.argtypes = [vp]
    hip.hipEventCreate.argtypes = [ctypes.POINTER(vp)]
    hip.hipEventRecord.argtypes = [vp, vp]
    hip.hipEventQuery.argtypes = [vp]
    hip.hipEventSynchronize.argtypes = [vp]
    n = 32 << 20
    srcs = [torch.rand(n, device="cuda") for _ in range(8)]
    out = torch.empty(n, device="cuda")
    op = nbx.host_to_dev_redop(0, 7, 1)
    sp = [t.data_ptr() for t in srcs]
    torch.cuda.synchronize()
    res = {"runtime": torch.version.hip}
    st, ev = vp(), vp()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) == 0
    assert hip.hipEventCreate(ctypes.byref(ev)) == 0
    t0 = time.perf_counter()
    for _ in range(200):   # ~50 us each
        nbx.reduce_multi([out.data_ptr()], sp, n, 7, op, 0, False, st.value)
    hip.hipEventRecord(ev, st)
    t1 = time.perf_counter()
    old = st.value
    assert hip.hipStreamDestroy(st) == 0
    t2 = time.perf_counter()
    pending = hip.hipEventQuery(ev) != 0
    hip.hipEventSynchronize(ev)
    t3 = time.perf_counter()
    st2 = vp()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(st2), 1) == 0
    res.update({"enqueue_ms": round((t1 - t0) * 1e3, 3), "destroy_ms": round((t2 - t1) * 1e3, 3),
                "work_pending_after_destroy": pending, "work_left_after_destroy_ms": round((t3 - t2) * 1e3, 3),
                "next_stream_reuses_handle": st2.value == old})
    hip.hipStreamDestroy(st2)
    handles, reuse = set(), 0
    for i in range(32):
        s = vp()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
        reuse += s.value in handles
        handles.add(s.value)
        for _ in range(4):
            nbx.reduce_multi([out.data_ptr()], sp, n, 7, op, 0, False, s.value)
        hip.hipStreamDestroy(s)
    torch.cuda.synchronize()
    res["cycles"], res["handle_reuse"] = 32, reuse
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
