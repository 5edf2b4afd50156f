#!/usr/bin/env python3
"""simple_traffic.py — HBM traffic of the multi-process Simple kernels
(VERDICT r3 next 3): the one-process rig (nbxDebugSimpleRun) with every rank's
workgroups in ONE dispatch (NBX_DEBUG_SIMPLE_FUSED=1, kSimpleFused), so
rocprofv3's PMC passes — which serialize dispatches and would deadlock the
per-rank launches that wait on each other — can count the call's FETCH_SIZE /
WRITE_SIZE. Config D's shape: fp32 sum AllReduce, `mib` MiB per rank, n ranks
sharing the GPU, direct or ring schedule. Prints one JSON line: device ms per
call and the byte models per dispatch (all ranks):
  algorithmic  n x (M read + M written)      (the user-visible bytes)
  staging      n x 2 x (M + 2 (n-1) M / n)   (direct and ring alike: each byte
               of a rank's input and output crosses staging once per hop)
usage: simple_traffic.py n mib ring(0|1) iters
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mib = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    ring = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    os.environ["NBX_DEBUG_SIMPLE_FUSED"] = "1"
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
    count = (mib << 20) // 4
    xs = [((torch.arange(count, device="cuda", dtype=torch.int32) * 7 + 13 * r) % 1024).to(torch.float32)
          for r in range(n)]
    ys = [torch.full((count,), -1.0, device="cuda") for _ in range(n)]
    send = (ctypes.c_void_p * n)(*[x.data_ptr() for x in xs])
    recv = (ctypes.c_void_p * n)(*[y.data_ptr() for y in ys])
    grid = min(128, 256 // n)   # the communicator's grid for n ranks sharing one GPU (mpTransportSettings)
    ms = ctypes.c_float()
    rc = lib.nbxDebugSimpleRun(n, 0, ring, count, 7, 0, send, recv, 0, grid, 64 << 10, 2, 1, iters, ctypes.byref(ms))
    exp = torch.zeros(count, device="cuda")
    for x in xs:
        exp += x
    exact = rc == 0 and all(torch.equal(y, exp) for y in ys)
    M = count * 4
    alg = n * 2 * M
    staging = n * 2 * (M + 2 * (n - 1) * M // n)
    print(json.dumps({"n": n, "MiB_per_rank": mib, "schedule": "ring" if ring else "direct", "rc": rc,
                      "exact": exact, "grid": grid, "dispatches": iters + 1, "ms_per_call": round(ms.value, 4),
                      "algorithmic_bytes_per_dispatch": alg, "staging_model_bytes_per_dispatch": staging,
                      "kernel": "kSimpleFused (every rank's workgroups in one dispatch)"}), flush=True)
    return 0 if exact else 1


if __name__ == "__main__":
    sys.exit(main())
