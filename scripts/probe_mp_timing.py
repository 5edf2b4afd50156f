#!/usr/bin/env python3
"""probe_mp_timing.py — per-call host enqueue time and device completion time
of multi-process Simple-path AllReduce, 2 ranks sharing GPU 0 (diagnostic)."""
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(uid, rank, n, q):
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    nbx.load_library()
    torch.cuda.set_device(0)
    comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid), rank)
    st = torch.cuda.current_stream().cuda_stream
    out = []
    for name, dt, op, tdt in (("i64max", 4, 2, torch.int64), ("f32sum", 7, 0, torch.float32),
                              ("i64sum", 4, 0, torch.int64), ("i32max", 2, 2, torch.int32)):
        cnt = (128 << 20) // torch.tensor([], dtype=tdt).element_size()
        x = torch.ones(cnt, dtype=tdt, device="cuda")
        y = torch.empty_like(x)
        for i in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            comm.all_reduce(x.data_ptr(), y.data_ptr(), cnt, dt, op, st)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            out.append({"what": name, "i": i, "enqueue_ms": round((t1 - t0) * 1e3, 3),
                        "complete_ms": round((t2 - t0) * 1e3, 3)})
    comm.destroy()
    q.put((rank, out))


if __name__ == "__main__":
    os.environ.setdefault("NBX_TIMEOUT_SEC", "60")
    from __graft_entry__ import _load_package
    nbx = _load_package()
    nbx.load_library()
    uid = bytes(nbx.get_unique_id())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=child, args=(uid, r, 2, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in ps:
        p.join()
    for row in res[0]:
        print(json.dumps(row))
