#!/usr/bin/env python3
"""probe_layout.py — does the placement of the 8 config-B inputs in HBM change
the reduce rate? (diagnostic, not a test).

Variants, all through the product C ABI (nbxReduceMulti, 8 x 256 MiB fp32 ->
256 MiB), interleaved over rounds:
  tensors      nine separate torch allocations (what bench.py does)
  skew:<d>     one slab, input k at k * (256 MiB + d) bytes, output after them
and two timing shapes for the bench's layout: one event pair around 10
back-to-back launches vs an event after every launch (bench.py's loop).
Prints one JSON line per variant.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N = 64 << 20          # fp32 elements per input
B = N * 4


def main():
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    lib = nbx.load_library()
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    op = nbx.host_to_dev_redop(0, 7, 1)
    rounds = int(os.environ.get("ROUNDS", "5"))

    def launcher(sp, dp):
        sa = (ctypes.c_void_p * 8)(*sp)
        da = (ctypes.c_void_p * 1)(dp)
        h = ctypes.c_void_p(st.cuda_stream)
        return lambda: lib.nbxReduceMulti(da, 1, sa, 8, N, 7, op, 0, 0, h)

    variants = {}
    g = torch.Generator(device="cuda").manual_seed(1)
    tens = [torch.rand(N, device="cuda", generator=g) for _ in range(8)]
    tout = torch.empty(N, device="cuda")
    variants["tensors"] = launcher([t.data_ptr() for t in tens], tout.data_ptr())
    skews = [0, 4096, 65536, 1 << 20, (1 << 20) + 4096, 3 << 20]
    slab = torch.empty(9 * B + 9 * max(skews) + 4096, dtype=torch.uint8, device="cuda")
    base = (slab.data_ptr() + 4095) // 4096 * 4096
    for d in skews:
        sp = [base + k * (B + d) for k in range(8)]
        dp = base + 8 * (B + d)
        variants[f"skew:{d}"] = launcher(sp, dp)
    slab.view(torch.float32)[: slab.numel() // 4].uniform_(-1, 1)
    addrs = {"tensors": [hex(t.data_ptr()) for t in tens] + [hex(tout.data_ptr())]}

    res = {k: [] for k in variants}
    res["tensors_event_per_launch"] = []
    for _ in range(rounds):
        for k, fn in variants.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(10):
                fn()
            e1.record(st)
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / 10)
        fn = variants["tensors"]
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(11)]
        evs[0].record(st)
        for i in range(10):
            fn()
            evs[i + 1].record(st)
        torch.cuda.synchronize()
        res["tensors_event_per_launch"].append(evs[0].elapsed_time(evs[10]) / 10)
    for k, v in res.items():
        v.sort()
        med = v[len(v) // 2]
        print(json.dumps({"variant": k, "med_ms": round(med, 4), "min_ms": round(v[0], 4),
                          "GBps": round(9 * B / (med * 1e-3) / 1e9, 1)}), flush=True)
    print(json.dumps({"addrs": addrs}), flush=True)


if __name__ == "__main__":
    main()
