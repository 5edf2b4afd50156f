#!/usr/bin/env python3
"""probe_mid_sizes.py — single-bucket reductions of mid-size buckets (1..64 MiB
per input, the config-C range) under each tile policy: auto, small tiles
(launch variant 1), big tiles (variant 2), one process; device time per call
from HIP events around back-to-back calls. Run it twice, with
NBX_DYNAMIC_TILES=0 and =1, to compare the big tile's static and dynamic
schedules. Not the bench. usage: probe_mid_sizes.py [--nsrc 8,4] [--dtypes fp16,fp32]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nsrc", default="8,4")
    ap.add_argument("--dtypes", default="fp16,fp32")
    ap.add_argument("--sizes", default="1,2,4,8,16,32,64")
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    lib = nbx.load_library()
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream().cuda_stream
    dts = {"fp16": (6, torch.float16, 2), "fp32": (7, torch.float32, 4)}
    for dname in args.dtypes.split(","):
        dt, tdt, esz = dts[dname]
        op = nbx.host_to_dev_redop(0, dt, 1)
        for nsrc in [int(x) for x in args.nsrc.split(",")]:
            for mib in [int(x) for x in args.sizes.split(",")]:
                n = (mib << 20) // esz
                srcs = [torch.rand(n, device="cuda").to(tdt) for _ in range(nsrc)]
                outs = {m: torch.empty_like(srcs[0]) for m in (0, 1, 2)}
                sa = (ctypes.c_void_p * nsrc)(*[t.data_ptr() for t in srcs])
                das = {m: (ctypes.c_void_p * 1)(o.data_ptr()) for m, o in outs.items()}
                iters = max(10, min(200, (4 << 30) // ((nsrc + 1) * (mib << 20))))
                times = {m: [] for m in (0, 1, 2)}
                for _ in range(args.rounds):
                    for m in (0, 1, 2):
                        nbx.set_launch_config(0, m)
                        for _ in range(3):
                            assert lib.nbxReduceMulti(das[m], 1, sa, nsrc, n, dt, op, 0, 0, ctypes.c_void_p(st)) == 0
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for _ in range(iters):
                            lib.nbxReduceMulti(das[m], 1, sa, nsrc, n, dt, op, 0, 0, ctypes.c_void_p(st))
                        e1.record()
                        torch.cuda.synchronize()
                        times[m].append(e0.elapsed_time(e1) / iters)
                nbx.set_launch_config(0, 0)
                same = torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
                row = {"dyn": os.environ.get("NBX_DYNAMIC_TILES", "1"), "dtype": dname, "nsrc": nsrc,
                       "MiB_per_input": mib, "identical": same}
                alg = (nsrc + 1) * (mib << 20)
                for m, name in ((0, "auto"), (1, "small"), (2, "big")):
                    ts = sorted(times[m])
                    ms = ts[len(ts) // 2]
                    row[name + "_us"] = round(ms * 1e3, 2)
                    row[name + "_GBps"] = round(alg / (ms * 1e-3) / 1e9, 1)
                print(json.dumps(row), flush=True)
                del srcs, outs


if __name__ == "__main__":
    main()
