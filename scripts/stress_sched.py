#!/usr/bin/env python3
"""stress_sched.py — randomized stress of the launch machinery added in round
2, on the GPU box: dynamic tile counters (per stream, host-tracked bases),
work-list table slots (event-tracked, graph-owned), kernel-argument fallbacks.
Mixes single-bucket reductions of 1-12 sources (big and small tiles,
multi-pass), batched calls of 1-400 buckets, four streams with cross-stream
dependencies, and graph captures replayed between eager calls. Inputs are
small integers in fp32, so every sum is exact and checked against torch.
Prints one JSON summary line; exits 1 on any mismatch."""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", type=int, default=600)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--dyn-min-tiles", type=int, default=0,
                    help="nbxDebugSetDynMinTiles for the run (1: every big-tile launch dynamic; 0: library default)")
    args = ap.parse_args(argv)
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    lib = nbx.load_library()
    prev_dyn = lib.nbxDebugSetDynMinTiles(args.dyn_min_tiles if args.dyn_min_tiles > 0 else 0)
    torch.cuda.set_device(0)
    rng = random.Random(args.seed)
    streams = [torch.cuda.Stream() for _ in range(4)]
    op = nbx.DevRedOpFull()
    pool = [torch.randint(-8, 8, (1 << 22,), device="cuda").float() for _ in range(12)]   # 16 MiB sources
    # the pool is written on the default stream; the four side streams do not
    # wait for it, so the first operations could read it half-written (the
    # r4a failure: every mismatch was among a run's first operations,
    # profiles/r2/stress_sched_seeds_r4b.jsonl)
    torch.cuda.synchronize()
    bad, checked, graphs, details = 0, 0, [], []
    t0 = time.time()

    def new_case(kind):
        if kind == "single":
            nsrc = rng.choice([1, 2, 3, 4, 5, 8, 8, 8, 12])
            n = rng.choice([rng.randint(1, 5000), rng.randint(1 << 18, 1 << 22)])
            off = rng.randint(0, (1 << 22) - n)
            srcs = [pool[(i * 5 + nsrc) % 12][off:off + n] for i in range(nsrc)]
            meta.update(kind="single", nsrc=nsrc, n=n, off=off)
            return [(srcs, torch.empty(n, device="cuda"))]
        nb = rng.choice([3, 17, 60, 200, 400])
        meta.update(kind="batch", buckets=nb)
        out = []
        for _ in range(nb):
            nsrc = rng.choice([2, 4, 8])
            n = rng.randint(1, 40000)
            off = rng.randint(0, (1 << 22) - n)
            out.append(([pool[(i * 7 + nsrc) % 12][off:off + n] for i in range(nsrc)], torch.empty(n, device="cuda")))
        return out

    def issue(case, s):
        if len(case) == 1 and rng.random() < 0.7:
            meta["call"] = "reduce_multi"
            srcs, o = case[0]
            nbx.reduce_multi([o.data_ptr()], [t.data_ptr() for t in srcs], o.numel(), 7, op, 0, False, s.cuda_stream)
        else:
            meta["call"] = "reduce_multi_batch"
            by = {}
            for srcs, o in case:   # batches take one source count's buckets at a time here too
                by.setdefault(len(srcs), []).append(([o.data_ptr()], [t.data_ptr() for t in srcs], o.numel()))
            for calls in by.values():
                nbx.reduce_multi_batch(calls, 7, op, 0, False, s.cuda_stream)

    def verify(case, m, phase):
        nonlocal bad, checked
        for k, (srcs, o) in enumerate(case):
            ref = srcs[0].clone()
            for t in srcs[1:]:
                ref += t
            checked += 1
            if not torch.equal(ref, o):
                bad += 1
                wrong = (ref != o).nonzero().flatten()
                i0 = int(wrong[0])
                details.append(dict(m, phase=phase, bucket=k, bucket_n=o.numel(), bucket_nsrc=len(srcs),
                                    src_off_bytes=[(t.data_ptr() % 4096) for t in srcs][:3],
                                    dst_off_bytes=o.data_ptr() % 4096, n_wrong=int(wrong.numel()),
                                    first_wrong=i0, last_wrong=int(wrong[-1]), ref=float(ref[i0]), got=float(o[i0]),
                                    unwritten=int((o[wrong] == 12345.0).sum())))

    live = []
    for i in range(args.ops):
        si = rng.randrange(4)
        s = streams[si]
        meta = {"op": i, "stream": si}
        case = new_case("single" if rng.random() < 0.6 else "batch")
        with torch.cuda.stream(s):
            for o in [o for _, o in case]:
                o.fill_(12345.0)
            r = rng.random()
            if r < 0.08:   # capture, replay now and once more later
                meta["graph"] = True
                g = torch.cuda.CUDAGraph()
                s.synchronize()
                with torch.cuda.graph(g, stream=s):
                    issue(case, s)
                g.replay()
                graphs.append((g, case, s, meta))
            else:
                issue(case, s)
            if rng.random() < 0.2:   # cross-stream dependency
                streams[rng.randrange(4)].wait_stream(s)
        live.append((case, meta))
        if len(live) >= 24:
            for st in streams:
                st.synchronize()
            for c, m in live:
                verify(c, m, "eager")
            live.clear()
    for st in streams:
        st.synchronize()
    for c, m in live:
        verify(c, m, "eager")
    for g, case, s, m in graphs:   # replay after everything else: the graph's table slot must be intact
        with torch.cuda.stream(s):
            for _, o in case:
                o.fill_(12345.0)
            g.replay()
        s.synchronize()
        verify(case, m, "final_replay")
    res = {"ops": args.ops, "outputs_checked": checked, "mismatches": bad, "graphs": len(graphs),
           "list_fallbacks": lib.nbxDebugBatchListSlots(0, 3), "list_slots_graph_owned": lib.nbxDebugBatchListSlots(0, 2),
           "seconds": round(time.time() - t0, 1), "bad_cases": details[:8]}
    del graphs
    lib.nbxDebugSetDynMinTiles(prev_dyn)
    res["dyn_min_tiles"] = args.dyn_min_tiles
    print(json.dumps(res), flush=True)
    return 0 if bad == 0 else 1, res


if __name__ == "__main__":
    sys.exit(main()[0])
