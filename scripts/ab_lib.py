#!/usr/bin/env python3
"""ab_lib.py — in-process A/B of two builds of libnbxccl.so on the config-B
workload (8 x 256 MiB fp32 sum): same buffers, same stream, interleaved
rounds; prints the median kernel time of each build (HIP events around 20
back-to-back calls). A library exporting sa_reduce8 (a bare standalone
kernel) can join the comparison. usage: ab_lib.py a.so b.so [c.so ...] [rounds]"""
import ctypes
import json
import sys

import torch


class DevRedOpFull(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("scalarArgIsPtr", ctypes.c_int32), ("scalarArg", ctypes.c_uint64)]


def load(path):
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    if hasattr(lib, "sa_reduce8"):   # a standalone kernel library: (dst, srcs[8], count, stream)
        g = lib.sa_reduce8
        g.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint64, ctypes.c_void_p]
        g.restype = ctypes.c_int
        return lambda D, nd, S, ns, n, dt, op, npre, post, st: g(D[0], S, n, st)
    f = lib.nbxReduceMulti
    f.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                  ctypes.c_size_t, ctypes.c_int, DevRedOpFull, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    f.restype = ctypes.c_int
    return f


def main():
    paths = [a for a in sys.argv[1:] if a.endswith(".so")]
    rest = [a for a in sys.argv[1:] if not a.endswith(".so")]
    rounds = int(rest[0]) if rest else 7
    fns = [load(p) for p in paths]
    n = 64 << 20
    g = torch.Generator(device="cuda").manual_seed(1)
    srcs = [torch.rand(n, device="cuda", generator=g) for _ in range(8)]
    out = torch.empty(n, device="cuda")
    S = (ctypes.c_void_p * 8)(*[t.data_ptr() for t in srcs])
    D = (ctypes.c_void_p * 1)(out.data_ptr())
    st = torch.cuda.current_stream()
    op = DevRedOpFull(0, 0, 0)
    times = [[] for _ in fns]
    for _ in range(rounds):
        for k, f in enumerate(fns):
            for _ in range(3):
                assert f(D, 1, S, 8, n, 7, op, 0, 0, st.cuda_stream) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(20):
                f(D, 1, S, 8, n, 7, op, 0, 0, st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 20)
    alg = 9 * n * 4
    for p, t in zip(paths, times):
        t = sorted(t)
        med = t[len(t) // 2]
        print(json.dumps({"lib": p, "median_ms": round(med, 5), "min_ms": round(t[0], 5),
                          "GBps": round(alg / med / 1e6, 1)}))


if __name__ == "__main__":
    main()
