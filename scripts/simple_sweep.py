#!/usr/bin/env python3
"""simple_sweep.py — tune the Simple protocol's kernels (nbx_simple.h) with
every rank in ONE process on one GPU (nbxDebugSimpleRun): AllReduce /
ReduceScatter of COUNT fp32 elements per rank over grid x slice x slots x
prefetch, direct and ring schedules; device ms per call and the algorithmic
bandwidth; the first config of each rank count is checked exactly.
usage: simple_sweep.py [n list] [MiB per rank] [configs: grid:sliceKiB:slots:prefetch,...]
Prints one JSON line per measurement."""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    lib = nbx.load_library()
    lib.nbxDebugSimpleRun.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_float)]
    lib.nbxDebugSimpleRun.restype = ctypes.c_int
    torch.cuda.set_device(0)
    ns = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [2]
    mib = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    cfgs = ([tuple(int(v) for v in c.split(":")) for c in sys.argv[3].split(",")] if len(sys.argv) > 3 else
            [(128, 64, 2, 1), (128, 64, 2, 0), (128, 128, 2, 1), (128, 256, 2, 1), (64, 256, 2, 1), (64, 512, 2, 1),
             (32, 1024, 2, 1), (128, 64, 4, 1), (64, 256, 4, 1)])
    count = (mib << 20) // 4
    for n in ns:
        xs = []
        for r in range(n):
            idx = torch.arange(count, device="cuda", dtype=torch.int32)
            xs.append(((idx * 7 + 13 * r) % 1024).to(torch.float32))
            del idx
        exp = torch.zeros(count, device="cuda")
        for x in xs:
            exp += x
        ys = [torch.empty(count, device="cuda") for _ in range(n)]
        send = (ctypes.c_void_p * n)(*[x.data_ptr() for x in xs])
        recv = (ctypes.c_void_p * n)(*[y.data_ptr() for y in ys])
        first = True
        for kind, kname in ((0, "allreduce"), (1, "reduce_scatter")):
            for ring in (0, 1):
                for grid, skib, slots, pre in cfgs:
                    if grid * n > 256:
                        continue
                    cnt = count if kind == 0 else count // n
                    for y in ys:
                        y.fill_(-1.0)
                    ms = ctypes.c_float()
                    rc = lib.nbxDebugSimpleRun(n, kind, ring, cnt, 7, 0, send, recv, 0, grid, skib << 10, slots, pre,
                                               3 if mib >= 256 else 10, ctypes.byref(ms))
                    ok = None
                    if rc == 0 and first:
                        ok = all(torch.equal(ys[r], exp if kind == 0 else exp[r * cnt:(r + 1) * cnt])
                                 for r in range(n))
                    alg = count * 4 / (ms.value * 1e-3) / 1e9 if rc == 0 and ms.value > 0 else None
                    print(json.dumps({"n": n, "op": kname, "algo": "ring" if ring else "direct", "grid": grid,
                                      "slice_KiB": skib, "slots": slots, "prefetch": pre, "rc": rc,
                                      "ms": round(ms.value, 4), "algbw_GBs": round(alg, 1) if alg else None,
                                      "exact": ok}), flush=True)
                    if rc != 0:
                        return 1
                first = False
        del xs, ys, exp
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
