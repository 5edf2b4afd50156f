#!/usr/bin/env python3
"""config_c_profile.py — config C (fp16 and bf16 ncclSum, 1..64 MiB per input,
nSrcs 2 and 8) through the product C ABI, laid out so that a
rocprofv3 kernel trace or PMC pass of this process can be cut into cases:
every case is bracketed by a marker dispatch (a 1-element fp32 3-source
nbxReduceMulti, a kernel no config-C case launches). Not the bench.

  run:        python scripts/config_c_profile.py [--iters N]           -> one JSON line per case (HIP events)
  summarize:  python scripts/config_c_profile.py --summarize CASES.jsonl TRACE.csv [PMC.csv ...]
              -> per case: rocprof device time per call (sum of the case's
                 dispatches / calls) next to the event time, and HBM bytes per
                 call from FETCH_SIZE (x2, gfx950) + WRITE_SIZE against the
                 algorithmic (nSrcs + 1) x bytes.
Cases: single-bucket calls (nbxReduceMulti) per size, and the whole 1..64 MiB
set as one nbxReduceMultiBatch call (auto routing).
"""
import argparse
import csv
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MARKER = "FnSumF<nbx::TyF32>, 3, 1>"
SIZES_MIB = (1, 2, 4, 8, 16, 32, 64)


def run(args):
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    lib = nbx.load_library()
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream().cuda_stream
    m_in = [torch.ones(4, device="cuda") for _ in range(3)]
    m_out = torch.empty(4, device="cuda")
    m_s = (ctypes.c_void_p * 3)(*[t.data_ptr() for t in m_in])
    m_d = (ctypes.c_void_p * 1)(m_out.data_ptr())
    m_op = nbx.host_to_dev_redop(0, 7, 1)

    def marker():
        assert lib.nbxReduceMulti(m_d, 1, m_s, 3, 1, 7, m_op, 0, 0, ctypes.c_void_p(st)) == 0

    for dt, name, tdt in ((6, "fp16", torch.float16), (9, "bf16", torch.bfloat16)):
        op = nbx.host_to_dev_redop(0, dt, 1)
        for nsrc in (2, 8):
            bufs = []
            for mib in SIZES_MIB:
                n = (mib << 20) // 2
                srcs = [(torch.rand(n, device="cuda") * 2 - 1).to(tdt) for _ in range(nsrc)]
                bufs.append((srcs, torch.empty_like(srcs[0]), n, mib))
            keep = []
            tasks = (nbx.ReduceTask * len(bufs))()
            singles = []
            for i, (ss, o, n, mib) in enumerate(bufs):
                da = (ctypes.c_void_p * 1)(o.data_ptr())
                sa = (ctypes.c_void_p * nsrc)(*[t.data_ptr() for t in ss])
                keep += [da, sa]
                tasks[i] = nbx.ReduceTask(da, 1, sa, nsrc, n)
                singles.append((da, sa, n, mib))
            cases = [(f"single_{mib}MiB", [(da, sa, n)], (nsrc + 1) * (mib << 20)) for da, sa, n, mib in singles]
            cases.append(("batch_1_64MiB", None, sum((nsrc + 1) * (m << 20) for m in SIZES_MIB)))
            for cname, calls, alg in cases:
                def one():
                    if calls is None:
                        assert lib.nbxReduceMultiBatch(tasks, len(bufs), dt, op, 0, 0, ctypes.c_void_p(st)) == 0
                    else:
                        for da, sa, n in calls:
                            assert lib.nbxReduceMulti(da, 1, sa, nsrc, n, dt, op, 0, 0, ctypes.c_void_p(st)) == 0
                for _ in range(2):
                    one()
                torch.cuda.synchronize()
                marker()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    one()
                e1.record()
                marker()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.iters
                print(json.dumps({"dtype": name, "nsrc": nsrc, "case": cname, "calls": args.iters,
                                  "alg_bytes_per_call": alg, "event_ms_per_call": round(ms, 5),
                                  "event_GBps": round(alg / (ms * 1e-3) / 1e9, 1)}), flush=True)
            del bufs, keep


def segments(rows, key):
    """Split dispatch rows (in order) at marker dispatches: the rows strictly
    between two consecutive markers form one timed segment."""
    out, cur, open_ = [], [], False
    for r in rows:
        if MARKER in r[key]:
            if open_:
                out.append(cur)
                cur, open_ = [], False
            else:
                cur, open_ = [], True
        elif open_:
            cur.append(r)
    return out


def summarize(args):
    cases = [json.loads(l) for l in open(args.summarize[0]) if l.startswith("{")]
    trace = list(csv.DictReader(open(args.summarize[1])))
    trace = [r for r in trace if "nbx::" in r["Kernel_Name"]]
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    seg = segments(trace, "Kernel_Name")
    pmc = {}
    for path in args.summarize[2:]:
        rows = list(csv.DictReader(open(path)))
        rows = [r for r in rows if "nbx::" in r["Kernel_Name"]]
        by = {}
        for r in rows:   # one row per (dispatch, counter)
            by.setdefault(int(r["Dispatch_Id"]), {"Kernel_Name": r["Kernel_Name"]})[r["Counter_Name"]] = float(
                r["Counter_Value"])
        disp = [by[k] for k in sorted(by)]
        for i, s in enumerate(segments(disp, "Kernel_Name")):
            for d in s:
                for c in ("FETCH_SIZE", "WRITE_SIZE"):
                    if c in d:
                        pmc.setdefault(i, {}).setdefault(c, 0.0)
                        pmc[i][c] += d[c]
    if len(seg) != len(cases):
        print(json.dumps({"error": f"{len(seg)} trace segments for {len(cases)} cases"}))
        return 1
    for i, (c, s) in enumerate(zip(cases, seg)):
        ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s)
        row = dict(c)
        row["rocprof_dispatches_per_call"] = round(len(s) / c["calls"], 2)
        row["rocprof_ms_per_call"] = round(ns / c["calls"] / 1e6, 5)
        row["rocprof_GBps"] = round(c["alg_bytes_per_call"] / (ns / c["calls"] * 1e-9) / 1e9, 1)
        row["kernels"] = sorted({r["Kernel_Name"].replace("void nbx::", "").split("(")[0] for r in s})
        if i in pmc and "FETCH_SIZE" in pmc[i] and "WRITE_SIZE" in pmc[i]:
            hbm = (2 * pmc[i]["FETCH_SIZE"] + pmc[i]["WRITE_SIZE"]) * 1024 / c["calls"]
            row["hbm_bytes_per_call"] = int(hbm)
            row["traffic_over_alg"] = round(hbm / c["alg_bytes_per_call"], 4)
        print(json.dumps(row))
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--summarize", nargs="+")
    args = ap.parse_args()
    if args.summarize:
        return summarize(args)
    run(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
