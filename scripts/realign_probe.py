#!/usr/bin/env python3
"""realign_probe.py — the library's realigning kernels at 256 MiB per input
(VERDICT r1 item 5), next to the aligned kernel on the same buffers: fp32 sum,
nSrcs in {2, 4, 8}, destination one element past the sources' alignment (so
every source is realigned), ITERS launches each. Prints one JSON line per case
(event-timed). Run it under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE /
TCC_HIT_sum,TCC_MISS_sum (separate passes) for the traffic ratio.
"""
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
    iters = int(os.environ.get("ITERS", "10"))
    mib = int(os.environ.get("MIB", "256"))
    n = (mib << 20) // 4
    st = torch.cuda.current_stream()
    op = nbx.host_to_dev_redop(nbx.ncclRedOp.ncclSum, nbx.ncclDataType.ncclFloat32, 1)
    srcs = [torch.rand(n + 64, device="cuda") for _ in range(8)]
    out = torch.empty(n + 64, device="cuda")
    for nsrc in (int(x) for x in os.environ.get("NSRCS", "8,4,2").split(",")):
        # aligned; every pointer one element off (shared misalignment: head
        # peel, body on a 16-B but not a 128-B boundary); destination one
        # element off (realigned sources)
        for label, soff, doff in (("aligned", 0, 0), ("shared_off+1", 1, 1), ("realigned_dst+1", 0, 1)):
            d = (ctypes.c_void_p * 1)(out.data_ptr() + 4 * doff)
            s = (ctypes.c_void_p * nsrc)(*[t.data_ptr() + 4 * soff for t in srcs[:nsrc]])
            call = lambda: lib.nbxReduceMulti(d, 1, s, nsrc, n, 7, op, 0, 0, ctypes.c_void_p(st.cuda_stream))
            call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(iters):
                call()
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / iters
            alg = (nsrc + 1) * n * 4
            print(json.dumps({"nsrc": nsrc, "MiB_per_input": mib, "case": label, "ms": round(ms, 4),
                              "GBps": round(alg / (ms * 1e-3) / 1e9, 1), "alg_bytes": alg}), flush=True)


if __name__ == "__main__":
    main()
