#!/usr/bin/env python3
"""ll128_stress.py — diagnostic for the LL128 protocol's line atomicity (not a
test of the suite): N processes (all on GPU 0, or one per GPU with
--per-gpu) run ITERS back-to-back LL128 collectives with inputs that change
every call (small integers, so any fold order gives the exact result) and
check every output. Mismatching elements are binned by the 8-byte word of the
payload line they travel in (--line-payload: 48 for the current 64-byte line,
the default; the original 128-byte-line run binned by 120): a torn
line — the flag visible before part of the payload — shows up as mismatches
concentrated in one part of the line (with 128-byte lines: words 0..7, the
first 64-byte half, profiles/r1/ll128_stress_128B.jsonl).

usage: python scripts/ll128_stress.py [--ranks 8] [--iters 300] [--count 131072]
           [--kind ar|rs] [--dtype 2] [--per-gpu]
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def child(uid_bytes, rank, n, args, q):
    try:
        import torch
        from __graft_entry__ import _load_package
        nbx = _load_package()
        nbx.load_library()
        dev = rank if args.per_gpu else 0
        torch.cuda.set_device(dev)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        st = torch.cuda.current_stream().cuda_stream
        tdt = {2: torch.int32, 7: torch.float32, 4: torch.int64}[args.dtype]
        eb = torch.tensor([], dtype=tdt).element_size()
        cnt = args.count
        total = cnt * n if args.kind == "rs" else cnt
        idx = torch.arange(total, device="cuda", dtype=torch.int64)
        words = torch.zeros(16, dtype=torch.int64)
        bad_calls = 0
        first_bad = None
        out = torch.empty(cnt, dtype=tdt, device="cuda")
        for it in range(args.iters):
            base = (idx * 7 + 13 * rank + 101 * it) % 1000
            x = base.to(tdt)
            exp_full = sum(((idx * 7 + 13 * r + 101 * it) % 1000) for r in range(n)).to(tdt)
            if args.kind == "rs":
                comm.reduce_scatter(x.data_ptr(), out.data_ptr(), cnt, args.dtype, 0, st)
                exp = exp_full[rank * cnt:(rank + 1) * cnt]
            else:
                comm.all_reduce(x.data_ptr(), out.data_ptr(), cnt, args.dtype, 0, st)
                exp = exp_full
            bad = (out != exp).nonzero().flatten()
            if bad.numel():
                bad_calls += 1
                w = ((bad * eb) % args.line_payload) // 8
                words += torch.bincount(w.cpu(), minlength=16)
                if first_bad is None:
                    e = int(bad[0])
                    first_bad = {"iter": it, "elem": e, "line": e * eb // args.line_payload, "n_bad": int(bad.numel()),
                                 "got": float(out[e]), "exp": float(exp[e])}
        torch.cuda.synchronize()
        comm.destroy()
        q.put((rank, "ok", {"bad_calls": bad_calls, "words": words.tolist(), "first_bad": first_bad}))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--count", type=int, default=131072)
    ap.add_argument("--kind", default="ar")
    ap.add_argument("--dtype", type=int, default=2)
    ap.add_argument("--per-gpu", action="store_true")
    ap.add_argument("--line-payload", type=int, default=48)
    args = ap.parse_args()
    os.environ.setdefault("NBX_TIMEOUT_SEC", "60")
    os.environ.setdefault("NBX_BOOTSTRAP_TIMEOUT", "60")
    os.environ.setdefault("NCCL_PROTO", "LL128")
    if not args.per_gpu:
        os.environ.setdefault("NBX_LL128_MAX_GRID", "16")
    from __graft_entry__ import _load_package
    nbx = _load_package()
    nbx.load_library()
    uid = nbx.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=child, args=(bytes(uid), r, args.ranks, args, q), daemon=True)
             for r in range(args.ranks)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(args.ranks):
            r, status, payload = q.get(timeout=600)
            res[r] = payload if status == "ok" else {"error": payload[-800:]}
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    print(json.dumps({"config": vars(args), "env": {k: os.environ.get(k) for k in
                                                    ("NCCL_PROTO", "NBX_LL128_MAX_GRID", "NBX_SYNC_MEM")},
                      "ranks": res}), flush=True)


if __name__ == "__main__":
    main()
