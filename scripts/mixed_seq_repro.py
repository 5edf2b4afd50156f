#!/usr/bin/env python3
"""mixed_seq_repro.py — replay test_multiprocess_ll_protocol's mixed sequence
(LL, LL128 one- and two-shot and Simple direct calls, back to back with no
host synchronisation) at N ranks sharing GPU 0, many iterations, and describe
every wrong output (tests/mp_diag.py): wrong-element count, their (block,
round, workgroup) cells, and what the wrong values equal — zero, a peer's raw
input, the fold without one source, or the previous iteration's output of that
call in that buffer position.

GPUTEST_r05: case 36 (int32 max, 1,000,003 elements, Simple direct) at 8
ranks returned wrong data on rank 0 with no error.

usage: mixed_seq_repro.py [--ranks 8] [--iters 10] [--cases 30:41] [--jitter]
Prints one JSON line: {"ranks", "iters", "calls", "mismatches": [...], "errors"}.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _cases():
    from tests.test_multiprocess_gpu import LL_CASES
    return LL_CASES


def _expected(oracle, case, i, n):
    """rank -> expected output (storage dtype), and the fold order per block."""
    import numpy as np
    from tests.test_multiprocess_gpu import _blocks, _ll_input, _ll_root
    kind, dtype, op, count, _ = case
    xs = [_ll_input(kind, dtype, count, n, r) for r in range(n)]
    devop, arg = oracle.host_to_dev_redop(op, dtype, n)
    st = oracle.NP_STORAGE[dtype]
    eb = np.dtype(st).itemsize
    kw = dict(n_pre_op_srcs=n, post_op=devop == 4)
    exp = {}
    if kind == "ar":
        full = np.empty(count, dtype=st)
        for c, (lo, hi) in enumerate(_blocks(count, eb, n)):
            if hi > lo:
                order = [(c + 1 + k) % n for k in range(n)]
                full[lo:hi] = oracle.reduce_multi([xs[j][lo:hi] for j in order], dtype, devop, arg, **kw)[0]
        exp = {r: full for r in range(n)}
    elif kind == "rs":
        for r in range(n):
            order = [(r + 1 + k) % n for k in range(n)]
            exp[r] = oracle.reduce_multi([xs[j][r * count:(r + 1) * count] for j in order], dtype, devop, arg,
                                         **kw)[0]
    else:
        root = _ll_root(i, n)
        order = [(root + 1 + k) % n for k in range(n)]
        exp[root] = oracle.reduce_multi([xs[j] for j in order], dtype, devop, arg, **kw)[0]
    return exp, xs


GUARD = 4096


def rank_main(uid_bytes, rank, n, iters, case_ids, jitter, q, fresh=False, skew=False, guard=False):
    try:
        import random

        import numpy as np
        import torch
        from oracle import oracle
        from tests.conftest import load_package
        from tests.test_multiprocess_gpu import _ll_input, _ll_root
        cases = _cases()
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        settings = comm_settings(nbx, comm)
        st = torch.cuda.current_stream().cuda_stream
        exp = {}
        for i in case_ids:
            e, _ = _expected(oracle, cases[i], i, n)
            if rank in e:
                exp[i] = np.ascontiguousarray(e[rank]).view(np.uint8)
        rng = random.Random(1234 + rank)
        bad = []
        guard_hits = []
        prev = {}
        calls = 0
        t0 = time.time()
        for it in range(iters):
            keep = []
            for i in case_ids:
                kind, dtype, op, count, shift = cases[i]
                x = _ll_input(kind, dtype, count, n, rank).view(np.uint8)
                G = GUARD if guard else 0   # guard bytes before and after (0xA5), checked after the iteration
                tx = torch.full((x.size + 16 + 2 * G,), 0xA5, dtype=torch.uint8, device="cuda")
                tx[G:G + x.size + 16] = 0
                tx[G + shift:G + shift + x.size] = torch.from_numpy(x.copy()).cuda()
                out_bytes = x.size // n if kind == "rs" else x.size
                ty = torch.full((out_bytes + 16 + 2 * G,), 0xA5, dtype=torch.uint8, device="cuda")
                ty[G:G + out_bytes + 16] = 0
                sp, rp = tx.data_ptr() + G + shift, ty.data_ptr() + G + shift
                if jitter and rng.random() < 0.3:
                    time.sleep(rng.random() * 0.004)
                if skew and rng.random() < 0.02:   # a rank stalls (first-launch code loading on a fresh box)
                    time.sleep(0.05 + rng.random() * 0.2)
                if kind == "ar":
                    comm.all_reduce(sp, rp, count, dtype, op, st)
                elif kind == "rs":
                    comm.reduce_scatter(sp, rp, count, dtype, op, st)
                else:
                    comm.reduce(sp, rp, count, dtype, op, _ll_root(i, n), st)
                calls += 1
                keep.append((i, ty, shift, out_bytes, tx, G))
            torch.cuda.synchronize()
            for i, ty, shift, nb, tx_, G in keep:
                if G:   # no byte outside [recv, recv + bytes) of the call's own slack may change
                    for name, t_ in (("send", tx_), ("recv", ty)):
                        lo, hi = t_[:G], t_[t_.numel() - G:]
                        if not (bool((lo == 0xA5).all()) and bool((hi == 0xA5).all())):
                            guard_hits.append({"it": it, "case": i, "buf": name,
                                               "before": int((lo != 0xA5).sum()), "after": int((hi != 0xA5).sum())})
                if i not in exp:
                    continue
                got = ty[G + shift:G + shift + nb].cpu().numpy().copy()
                if not np.array_equal(got, exp[i]):
                    bad.append({"it": it, "case": i, "got": got, "prev": prev.get(i)})
                prev[i] = got
            del keep
            if rank == 0 and (it % 5 == 0 or it == iters - 1):   # progress (a silent GPU run is taken for hung)
                print(f"[repro] iteration {it + 1}/{iters}, {time.time() - t0:.1f} s, rank 0 bad calls {len(bad)}",
                      file=sys.stderr, flush=True)
            if fresh:   # every buffer a fresh allocation next iteration (as iteration 0 of the GPU test)
                torch.cuda.empty_cache()
        err = comm.async_error()
        comm.destroy()
        q.put((rank, "ok", {"bad": bad, "guard_hits": guard_hits, "calls": calls, "async_error": err,
                            "settings": settings,
                            "s": time.time() - t0, "iters_done": it + 1}))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def comm_settings(nbx, comm):
    from tests import mp_diag
    return mp_diag.comm_settings(nbx, comm)


def diagnose(oracle, n, case_id, rank, got_u8, prev_u8, settings):
    from tests import mp_diag
    from tests.test_multiprocess_gpu import _ll_input, _ll_root
    kind, dtype, op, count, _ = _cases()[case_id]
    xs = [_ll_input(kind, dtype, count, n, r) for r in range(n)]
    return mp_diag.diagnose_collective(oracle, kind, dtype, op, count, n, rank, got_u8, xs, settings, prev_u8,
                                       root=_ll_root(case_id, n))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cases", default="0:41")
    ap.add_argument("--jitter", action="store_true")
    ap.add_argument("--fresh", action="store_true", help="torch.cuda.empty_cache() after every iteration")
    ap.add_argument("--skew", action="store_true", help="ranks stall 50-250 ms now and then")
    ap.add_argument("--guard", action="store_true", help="4 KiB 0xA5 guards around every buffer, checked")
    args = ap.parse_args()
    lo, hi = (int(x) for x in args.cases.split(":"))
    case_ids = list(range(lo, min(hi, len(_cases()))))
    os.environ.setdefault("NBX_BOOTSTRAP_TIMEOUT", "60")
    os.environ.setdefault("NBX_TIMEOUT_SEC", "60")
    os.environ.setdefault("NBX_LL128_MAX_GRID", "16")
    from oracle import oracle
    oracle.build()
    from tests.conftest import load_package
    nbx = load_package()
    nbx.load_library()
    n = args.ranks
    uid = nbx.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=rank_main, args=(bytes(uid), r, n, args.iters, case_ids, args.jitter, q, args.fresh,
                                                     args.skew, args.guard), daemon=True)
             for r in range(n)]
    for p in procs:
        p.start()
    res, errors = {}, []
    import queue as _queue
    t_start = time.time()
    try:
        for _ in range(n):
            while True:   # a heartbeat every 30 s (a fresh box's first torch import takes minutes)
                try:
                    rank, status, payload = q.get(timeout=30)
                    break
                except _queue.Empty:
                    print(f"[repro] waiting for the ranks, {time.time() - t_start:.0f} s", file=sys.stderr, flush=True)
                    if time.time() - t_start > 900:
                        raise
            if status != "ok":
                errors.append({"rank": rank, "error": payload[-3000:]})
            else:
                res[rank] = payload
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
    mism = []
    for r, pl in sorted(res.items()):
        for b in pl["bad"][:6]:
            d = diagnose(oracle, n, b["case"], r, b["got"], b["prev"], pl["settings"])
            mism.append({"rank": r, "it": b["it"], "case": b["case"], "call": list(_cases()[b["case"]]), **d})
    out = {"ranks": n, "iters": args.iters, "cases": args.cases, "jitter": args.jitter, "fresh": args.fresh,
           "skew": args.skew, "iters_done": {r: pl.get("iters_done") for r, pl in res.items()},
           "env": {k: v for k, v in os.environ.items() if k.startswith(("NBX_", "NCCL_"))},
           "calls": sum(pl["calls"] for pl in res.values()),
           "bad_calls": sum(len(pl["bad"]) for pl in res.values()),
           "bad_per_rank": {r: len(pl["bad"]) for r, pl in res.items()},
           "guard_hits": {r: pl["guard_hits"][:4] for r, pl in res.items() if pl.get("guard_hits")},
           "async_errors": {r: pl["async_error"] for r, pl in res.items() if pl["async_error"]},
           "settings": res[min(res)]["settings"] if res else None,
           "seconds": max((pl["s"] for pl in res.values()), default=None),
           "mismatches": mism, "errors": errors}
    print(json.dumps(out, default=str), flush=True)
    return 1 if (mism or errors or out["guard_hits"]) else 0


if __name__ == "__main__":
    sys.exit(main())
