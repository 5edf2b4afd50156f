#!/usr/bin/env python3
"""probe_batch_eager.py — per-call host enqueue time and per-call wall time of
eager nbxReduceMultiBatch calls (work list vs kernel-argument tables), one
process, on the GPU box. Not the bench. Env NBX_BATCH_TABLE_DEVICE selects the
work list's table memory (1 device via the large BAR, 0 pinned host)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    lib = nbx.load_library()
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream().cuda_stream
    dt, nsrc = 6, 2
    for sname, sizes in (("16x1MiB", [1 << 20] * 16), ("128x64KiB", [64 << 10] * 128)):
        bufs = []
        for b in sizes:
            n = b // 2
            srcs = [torch.rand(n, device="cuda").half() for _ in range(nsrc)]
            bufs.append((srcs, torch.empty_like(srcs[0]), n))
        tasks = (nbx.ReduceTask * len(bufs))()
        keep = []
        for i, (ss, o, n) in enumerate(bufs):
            da = (ctypes.c_void_p * 1)(o.data_ptr())
            sa = (ctypes.c_void_p * nsrc)(*[t.data_ptr() for t in ss])
            keep += [da, sa]
            tasks[i] = nbx.ReduceTask(da, 1, sa, nsrc, n)
        op = nbx.host_to_dev_redop(0, dt, 1)
        for mode in (1, 0, 1):
            lib.nbxDebugSetBatchMode(mode)
            for _ in range(5):
                lib.nbxReduceMultiBatch(tasks, len(bufs), dt, op, 0, 0, ctypes.c_void_p(st))
            torch.cuda.synchronize()
            iters = 200
            t0 = time.perf_counter()
            enq = []
            for _ in range(iters):
                a = time.perf_counter()
                lib.nbxReduceMultiBatch(tasks, len(bufs), dt, op, 0, 0, ctypes.c_void_p(st))
                enq.append(time.perf_counter() - a)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            enq.sort()
            print(json.dumps({"set": sname, "mode": "list" if mode else "kernarg",
                              "table_device": os.environ.get("NBX_BATCH_TABLE_DEVICE", "1"),
                              "enqueue_us_med": round(enq[len(enq) // 2] * 1e6, 2),
                              "enqueue_us_max": round(enq[-1] * 1e6, 2),
                              "wall_us_per_call": round((t2 - t0) / iters * 1e6, 2),
                              "free_slots": lib.nbxDebugBatchListSlots(0, 0),
                              "inflight_slots": lib.nbxDebugBatchListSlots(0, 1),
                              "fallbacks_total": lib.nbxDebugBatchListSlots(0, 3)}), flush=True)
        del bufs


if __name__ == "__main__":
    main()
