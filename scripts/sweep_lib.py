#!/usr/bin/env python3
"""Measurements through the product C ABI (libnbxccl.so), one process, on the
GPU box. Not the bench: feeds DESIGN.md and the launch-default choice.

  knobs   config B (8 x 256 MiB fp32 sum) under launch settings, interleaved rounds
  sweep   config C: fp16 / bf16 (and fp32, fp8) sum, nSrcs in {2, 8}, 1..64 MiB per input
  e2e     host-staged path: pinned host -> hipMemcpy H2D -> reduce -> D2H (BASELINE asks for it)
  small   latency of small buckets (4 KiB .. 1 MiB), nSrcs 2
  tiles   single-bucket tile choice: auto / small (U=1, 8 per CU) / big per nSrcs, dtype, size
  mixed   mixed pointer alignment (element kernel) vs shared alignment, 2 / 8 sources
  batch   config C bucket sets through nbxReduceMultiBatch vs one nbxReduceMulti per bucket

Prints one JSON object per line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def gbps(nbytes, ms):
    return nbytes / (ms * 1e-3) / 1e9


def timed(torch, fn, iters, warm=2):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="knobs,pipe,sweep,e2e,small")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--tiles-nsrc", type=lambda v: [int(x) for x in v.split(",")], default=[1, 2, 3, 4, 6, 8])
    ap.add_argument("--batch-sets", default="", help="comma-separated subset of the batch bucket sets")
    ap.add_argument("--tiles-settings", default="0:0,0:1,4:1,0:2,2:2", help="blocksPerCU:variant,...")
    args = ap.parse_args()
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    nbx.load_library()
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream().cuda_stream
    what = set(args.what.split(","))

    def op_for(dt):
        return nbx.host_to_dev_redop(0, dt, 1)

    if "knobs" in what:
        n = 64 << 20
        srcs = [torch.rand(n, device="cuda") for _ in range(8)]
        out = torch.empty(n, device="cuda")
        sp = [t.data_ptr() for t in srcs]
        op = op_for(7)
        settings = [(0, 0), (1, 2), (2, 2), (4, 2), (8, 1), (4, 1), (16, 1)]
        res = {s: [] for s in settings}
        for _ in range(args.rounds):
            for s in settings:
                nbx.set_launch_config(*s)
                res[s].append(timed(torch, lambda: nbx.reduce_multi([out.data_ptr()], sp, n, 7, op, 0, False, st), 10))
        nbx.set_launch_config(0, 0)
        for s, v in res.items():
            v.sort()
            print(json.dumps({"what": "knobs", "blocks_per_cu": s[0], "variant": s[1], "med_ms": round(v[len(v) // 2], 4),
                              "GBps": round(gbps(9 * n * 4, v[len(v) // 2]), 1)}), flush=True)
        del srcs, out

    if "pipe" in what:
        # in-process A/B of the big-tile kernel: software-pipelined (variant 2) vs not (3)
        for nsrc in (2, 4, 8):
            n = 64 << 20
            srcs = [torch.rand(n, device="cuda") for _ in range(nsrc)]
            out = torch.empty(n, device="cuda")
            sp = [t.data_ptr() for t in srcs]
            op = op_for(7)
            res = {2: [], 3: []}
            for _ in range(args.rounds):
                for v in (2, 3):
                    nbx.set_launch_config(0, v)
                    res[v].append(timed(torch, lambda: nbx.reduce_multi([out.data_ptr()], sp, n, 7, op, 0, False, st), 10))
            nbx.set_launch_config(0, 0)
            for v, t in res.items():
                t.sort()
                print(json.dumps({"what": "pipe", "nsrc": nsrc, "variant": "pipelined" if v == 2 else "plain",
                                  "med_ms": round(t[len(t) // 2], 4),
                                  "GBps": round(gbps((nsrc + 1) * n * 4, t[len(t) // 2]), 1)}), flush=True)
            del srcs, out

    if "sweep" in what:
        for dt, name, tdt in ((6, "fp16", torch.float16), (9, "bf16", torch.bfloat16), (7, "fp32", torch.float32),
                              (10, "fp8e4m3", torch.uint8)):
            for nsrc in (2, 8):
                for mib in (1, 2, 4, 8, 16, 32, 64):
                    esz = torch.tensor([], dtype=tdt).element_size()
                    n = (mib << 20) // esz
                    if tdt == torch.uint8:
                        srcs = [torch.randint(0, 120, (n,), dtype=torch.uint8, device="cuda") for _ in range(nsrc)]
                    else:
                        srcs = [torch.rand(n, device="cuda").to(tdt) for _ in range(nsrc)]
                    out = torch.empty_like(srcs[0])
                    sp = [t.data_ptr() for t in srcs]
                    op = op_for(dt)
                    iters = max(5, min(200, (256 << 20) // (mib << 20) * 4))
                    ts = sorted(timed(torch, lambda: nbx.reduce_multi([out.data_ptr()], sp, n, dt, op, 0, False, st),
                                      iters) for _ in range(args.rounds))
                    ms = ts[len(ts) // 2]   # median of rounds
                    print(json.dumps({"what": "sweep", "dtype": name, "nsrc": nsrc, "MiB_per_input": mib,
                                      "ms": round(ms, 5), "GBps": round(gbps((nsrc + 1) * n * esz, ms), 1)}),
                          flush=True)
                    del srcs, out

    if "e2e" in what:
        # host-staged: sources start in pinned host memory (the proxy/net staging
        # buffers), result returns to pinned host memory
        for nsrc, mib in ((2, 4), (8, 256), (2, 256), (2, 1), (8, 16), (2, 64)):
            n = (mib << 20) // 4
            hs = [torch.rand(n).pin_memory() for _ in range(nsrc)]
            ho = torch.empty(n).pin_memory()
            ds = [torch.empty(n, device="cuda") for _ in range(nsrc)]
            do = torch.empty(n, device="cuda")
            sp = [t.data_ptr() for t in ds]
            op = op_for(7)

            def run():
                for h, d in zip(hs, ds):
                    d.copy_(h, non_blocking=True)
                nbx.reduce_multi([do.data_ptr()], sp, n, 7, op, 0, False, st)
                ho.copy_(do, non_blocking=True)

            ms = timed(torch, run, 5 if mib > 16 else 20)
            kms = timed(torch, lambda: nbx.reduce_multi([do.data_ptr()], sp, n, 7, op, 0, False, st), 10)
            alg = (nsrc + 1) * n * 4
            # host entry point (blocking call; wall clock): the pipelined staging
            # ring, and zero-copy (the kernel reads / writes the pinned buffers)
            hp = [h.data_ptr() for h in hs]
            reps = 3 if mib > 16 else 20
            modes = {}
            for mode in ("staged", "zerocopy"):
                os.environ["NBX_HOST_MODE"] = mode
                nbx.reduce_multi_host([ho.data_ptr()], hp, n, 7, op, 0, False, st)
                t0 = time.perf_counter()
                for _ in range(reps):
                    nbx.reduce_multi_host([ho.data_ptr()], hp, n, 7, op, 0, False, st)
                modes[mode] = (time.perf_counter() - t0) * 1e3 / reps
            os.environ.pop("NBX_HOST_MODE")
            pms = modes["staged"]
            zms = modes["zerocopy"]
            print(json.dumps({"what": "e2e", "nsrc": nsrc, "MiB_per_input": mib, "e2e_ms": round(ms, 4),
                              "e2e_alg_GBps": round(gbps(alg, ms), 1), "kernel_ms": round(kms, 4),
                              "kernel_GBps": round(gbps(alg, kms), 1),
                              "pipelined_host_ms": round(pms, 4), "pipelined_host_alg_GBps": round(gbps(alg, pms), 1),
                              "zerocopy_ms": round(zms, 4), "zerocopy_alg_GBps": round(gbps(alg, zms), 1),
                              "pcie_bytes": alg}), flush=True)
            del hs, ho, ds, do

    if "tiles" in what:
        for dt, name, tdt in ((6, "fp16", torch.float16), (7, "fp32", torch.float32)):
            for nsrc in args.tiles_nsrc:
                for mib in (4, 16, 64, 256):
                    if nsrc * mib > 2048:
                        continue
                    esz = torch.tensor([], dtype=tdt).element_size()
                    n = (mib << 20) // esz
                    srcs = [torch.rand(n, device="cuda").to(tdt) for _ in range(nsrc)]
                    out = torch.empty_like(srcs[0])
                    sp = [t.data_ptr() for t in srcs]
                    op = op_for(dt)
                    settings = [tuple(int(v) for v in x.split(":")) for x in args.tiles_settings.split(",")]
                    res = {x: [] for x in settings}
                    for _ in range(args.rounds):
                        for x in settings:
                            nbx.set_launch_config(*x)
                            res[x].append(timed(torch, lambda: nbx.reduce_multi([out.data_ptr()], sp, n, dt, op, 0,
                                                                                False, st), 10))
                    nbx.set_launch_config(0, 0)
                    alg = (nsrc + 1) * n * esz
                    row = {"what": "tiles", "dtype": name, "nsrc": nsrc, "MiB_per_input": mib}
                    for x, v in res.items():
                        v.sort()
                        row[f"bpc{x[0]}_v{x[1]}_GBps"] = round(gbps(alg, v[len(v) // 2]), 1)
                    print(json.dumps(row), flush=True)
                    del srcs, out

    if "mixed" in what:
        for dt, name, tdt in ((7, "fp32", torch.float32), (6, "fp16", torch.float16)):
            for nsrc in [int(x) for x in os.environ.get("NBX_SWEEP_NSRCS", "2,3,4,8").split(",")]:
                esz = torch.tensor([], dtype=tdt).element_size()
                mib = int(os.environ.get("NBX_SWEEP_MIB", "64"))
                n = (mib << 20) // esz
                raw = [torch.rand(n + 16, device="cuda").to(tdt) for _ in range(nsrc)]
                out = torch.empty(n + 16, dtype=tdt, device="cuda")
                op = op_for(dt)
                row = {"what": "mixed", "dtype": name, "nsrc": nsrc, "MiB_per_input": mib}
                for label, doff in (("aligned", 0), ("dst_off_1elt", 1)):
                    sp = [t.data_ptr() for t in raw]
                    dp = out.data_ptr() + doff * esz
                    ts = sorted(timed(torch, lambda: nbx.reduce_multi([dp], sp, n, dt, op, 0, False, st), 10)
                                for _ in range(args.rounds))
                    row[label + "_GBps"] = round(gbps((nsrc + 1) * n * esz, ts[len(ts) // 2]), 1)
                print(json.dumps(row), flush=True)
                del raw, out

    if "batch" in what:
        # bucket sets (MiB per input): 16 x 1 MiB, 64 x 256 KiB, the mixed 1..64 MiB sweep
        sets = {"16x1MiB": [1 << 20] * 16, "64x256KiB": [256 << 10] * 64, "128x64KiB": [64 << 10] * 128,
                "mixed_1_64MiB": [m << 20 for m in (1, 2, 4, 8, 16, 32, 64)],
                "4x16MiB": [16 << 20] * 4, "1x64MiB": [64 << 20], "1x256MiB": [256 << 20]}
        only = set(args.batch_sets.split(",")) if args.batch_sets else set(sets)
        for dt, name, tdt in ((6, "fp16", torch.float16), (9, "bf16", torch.bfloat16), (7, "fp32", torch.float32)):
            for nsrc in (2, 8):
                for sname, sizes in sets.items():
                    if sname not in only or (dt == 7) != (sname == "1x256MiB"):
                        continue   # fp32 only for the config-B-sized bucket
                    bufs = []
                    esz = torch.tensor([], dtype=tdt).element_size()
                    for b in sizes:
                        n = b // esz
                        srcs = [torch.rand(n, device="cuda").to(tdt) for _ in range(nsrc)]
                        bufs.append((srcs, torch.empty_like(srcs[0]), n))
                    calls = [([o.data_ptr()], [t.data_ptr() for t in ss], n) for ss, o, n in bufs]
                    alg = sum((nsrc + 1) * b for b in sizes)
                    op = op_for(dt)
                    iters = max(5, min(100, (2 << 30) // alg))
                    lib = nbx.load_library()
                    keep = []
                    tasks = (nbx.ReduceTask * len(calls))()
                    singles = []
                    for i, (d, s_, n) in enumerate(calls):
                        da = (ctypes.c_void_p * 1)(*d)
                        sa = (ctypes.c_void_p * nsrc)(*s_)
                        keep += [da, sa]
                        tasks[i] = nbx.ReduceTask(da, 1, sa, nsrc, n)
                        singles.append((da, sa, n))

                    def enqueue(mode, stream):
                        # raw ctypes calls on prebuilt arrays: the GPU time, not Python's
                        if mode == "single":
                            for da, sa, n in singles:
                                lib.nbxReduceMulti(da, 1, sa, nsrc, n, dt, op, 0, 0, ctypes.c_void_p(stream))
                        else:
                            lib.nbxReduceMultiBatch(tasks, len(calls), dt, op, 0, 0, ctypes.c_void_p(stream))

                    res = {}
                    for mode in ("single", "batch_auto", "batch_kernarg", "batch_all"):
                        nbx.set_launch_config(0, 1 if mode == "batch_all" else 0)
                        # batch_kernarg: the kernel-argument tables instead of work lists
                        lib.nbxDebugSetBatchMode(0 if mode == "batch_kernarg" else 1)
                        # eager (host launch rate included) and graph-replayed (device time)
                        t = [timed(torch, lambda: enqueue(mode, st), iters) for _ in range(args.rounds)]
                        g = torch.cuda.CUDAGraph()
                        cs = torch.cuda.Stream()
                        with torch.cuda.stream(cs):
                            enqueue(mode, cs.cuda_stream)
                            torch.cuda.synchronize()
                            with torch.cuda.graph(g, stream=cs):
                                for _ in range(10):
                                    enqueue(mode, cs.cuda_stream)
                        tg = [timed(torch, g.replay, max(1, iters // 10)) / 10 for _ in range(args.rounds)]
                        nbx.set_launch_config(0, 0)
                        lib.nbxDebugSetBatchMode(1)
                        t.sort()
                        tg.sort()
                        res[mode] = t[len(t) // 2]
                        res[mode + "_graph"] = tg[len(tg) // 2]
                        del g
                    print(json.dumps({"what": "batch", "dtype": name, "nsrc": nsrc, "set": sname,
                                      "n_buckets": len(sizes), "alg_bytes": alg,
                                      **{f"{m}_ms": round(v, 4) for m, v in res.items()},
                                      **{f"{m}_GBps": round(gbps(alg, v), 1) for m, v in res.items()}}), flush=True)
                    del bufs

    if "small" in what:
        for kib in (4, 16, 64, 256, 1024):
            n = (kib << 10) // 4
            srcs = [torch.rand(n, device="cuda") for _ in range(2)]
            out = torch.empty_like(srcs[0])
            sp = [t.data_ptr() for t in srcs]
            op = op_for(7)
            ms = timed(torch, lambda: nbx.reduce_multi([out.data_ptr()], sp, n, 7, op, 0, False, st), 200, warm=20)
            print(json.dumps({"what": "small", "KiB_per_input": kib, "us_per_call": round(ms * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
