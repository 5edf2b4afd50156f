#!/usr/bin/env python3
"""probe_uc_bandwidth.py — what uncached (MTYPE UC, hipDeviceMallocUncached)
device memory costs a local streaming kernel, since the Simple protocol's
staging lives there (nbx_simple.h): the production copy kernel
(nbxReduceMulti, one source) between coarse-grained (hipMalloc) and uncached
buffers in all four directions, and the 8:1 fold reading from uncached
sources, one GPU, HIP events. Prints one JSON line."""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    nbx.load_library()
    torch.cuda.set_device(0)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n = (mib << 20) // 4
    st = torch.cuda.current_stream()
    op = nbx.host_to_dev_redop(0, 7, 1)

    def uc():
        p = ctypes.c_void_p()
        assert hip.hipExtMallocWithFlags(ctypes.byref(p), n * 4, 0x3) == 0
        return p.value

    bufs = {"coarse_a": torch.rand(n, device="cuda").data_ptr(), "coarse_b": torch.empty(n, device="cuda").data_ptr()}
    keep = [torch.rand(n, device="cuda") for _ in range(9)]
    ucs = [uc() for _ in range(9)]
    nbx.reduce_multi([ucs[0]], [keep[0].data_ptr()], n, 7, op, 0, False, st.cuda_stream)   # fill
    bufs["coarse_a"], bufs["coarse_b"] = keep[0].data_ptr(), keep[1].data_ptr()

    def timed(dsts, srcs, reps=10):
        for _ in range(2):
            nbx.reduce_multi(dsts, srcs, n, 7, op, 0, False, st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            nbx.reduce_multi(dsts, srcs, n, 7, op, 0, False, st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        return round((len(srcs) + len(dsts)) * n * 4 / (ms * 1e-3) / 1e9, 1)

    out = {"MiB_per_buffer": mib, "unit": "GB/s (algorithmic bytes / kernel time)"}
    out["copy_coarse_to_coarse"] = timed([keep[1].data_ptr()], [keep[0].data_ptr()])
    out["copy_uc_to_coarse"] = timed([keep[1].data_ptr()], [ucs[0]])
    out["copy_coarse_to_uc"] = timed([ucs[1]], [keep[0].data_ptr()])
    out["copy_uc_to_uc"] = timed([ucs[1]], [ucs[0]])
    for i in range(1, 8):
        nbx.reduce_multi([ucs[i]], [keep[i].data_ptr()], n, 7, op, 0, False, st.cuda_stream)
    out["fold8_coarse_srcs"] = timed([keep[8].data_ptr()], [k.data_ptr() for k in keep[:8]], 5)
    out["fold8_uc_srcs"] = timed([keep[8].data_ptr()], ucs[:8], 5)
    out["fold8_uc_srcs_uc_dst"] = timed([ucs[8]], ucs[:8], 5)
    torch.cuda.synchronize()
    for p in ucs:
        hip.hipFree(p)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
