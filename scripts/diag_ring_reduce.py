#!/usr/bin/env python3
"""Diagnose NCCL_ALGO=Ring Reduce on the multi-process communicator (2 ranks,
one GPU): which elements come out wrong, alone and after a ring AllReduce."""
import json
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(uid, rank, n, q, prior):
    import torch
    os.environ["NCCL_ALGO"] = "Ring"
    os.environ["NCCL_PROTO"] = "Simple"
    from __graft_entry__ import _load_package
    nbx = _load_package()
    nbx.load_library()
    torch.cuda.set_device(0)
    comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid), rank)
    st = torch.cuda.current_stream().cuda_stream
    out = {}
    if prior:
        x = torch.ones(1 << 18, device="cuda")
        y = torch.empty_like(x)
        comm.all_reduce(x.data_ptr(), y.data_ptr(), x.numel(), 7, 0, st)
        torch.cuda.synchronize()
        out["prior_ok"] = bool((y == n).all())
    for it, cnt in enumerate([1024, 1024, 4096, 1 << 18]):
        idx = torch.arange(cnt, device="cuda", dtype=torch.float32)
        x = torch.remainder(idx * 5 + 3 * rank + it, 509)
        y = torch.full((cnt,), -1.0, device="cuda")
        comm.reduce(x.data_ptr(), y.data_ptr() if rank == 0 else 0, cnt, 7, 0, 0, st)
        torch.cuda.synchronize()
        if rank == 0:
            want = sum(torch.remainder(idx * 5 + 3 * r + it, 509) for r in range(n))
            bad = (y != want).nonzero().flatten().tolist()
            out[f"call{it}_{cnt}"] = {"n_bad": len(bad), "first": bad[:40],
                                      "got": [float(y[i]) for i in bad[:8]], "want": [float(want[i]) for i in bad[:8]],
                                      "own": [float(x[i]) for i in bad[:8]]}
    comm.destroy()
    q.put((rank, out))


def main():
    from __graft_entry__ import _load_package
    nbx = _load_package()
    ctx = mp.get_context("spawn")
    for prior in (False, True):
        uid = bytes(nbx.get_unique_id())
        q = ctx.Queue()
        ps = [ctx.Process(target=child, args=(uid, r, 2, q, prior), daemon=True) for r in range(2)]
        for p in ps:
            p.start()
        res = dict(q.get(timeout=120) for _ in range(2))
        for p in ps:
            p.join(30)
        print(json.dumps({"prior_allreduce": prior, "root": res[0]}), flush=True)


if __name__ == "__main__":
    os.environ.setdefault("NBX_TIMEOUT_SEC", "30")
    os.environ.setdefault("NBX_SIMPLE_MAX_GRID", "16")
    main()
