#!/usr/bin/env python3
"""set_thresholds.py — protocol thresholds of the multi-rank communicators
from a bench line's measured sweep, instead of tuning them
by hand on the shared-GPU rig.

Input: a bench.py output (a file of JSON lines; the last line with a
`collective` object is used) from an N > 1 run. Its `collective.protocol_sweep`
holds, per message size, the max-over-ranks µs per AllReduce of every protocol
forced in turn (LL and LL128 with their buffers enlarged to 16 MiB; "LL128"
switches to the two-shot kernel above the one-shot limit when n > 2,
"LL128_oneshot" never does; every size checked exact by the leg).

Rule: walking the sizes upward, the protocol in use stays until another one is
faster by more than a hysteresis margin (default 5 %); ties and small wins keep
the current one (fewer switches, no flapping on noise). The ladder is
LL -> LL128 -> Simple (a protocol once left is not re-entered: buffer limits
are upper bounds), and a threshold is the largest swept size its protocol
still carries. Emitted (as NBX_* environment settings, read at communicator
creation, comm_mp_init.cc):
  NBX_LL_MAX_BYTES         largest size carried by LL (0 sizes: 1 KiB minimum)
  NBX_LL128_MAX_BYTES      largest size carried by LL128 (0 = LL128 never wins)
  NBX_LL128_ONESHOT_MAX    (n > 2) largest LL128 size at which one-shot is not
                           beaten by two-shot by more than the margin
  NCCL_ALGO                "Ring" when the ring's 1 GiB AllReduce beats the
                           direct schedule's by more than the margin
  NBX_CLIQUE_SIMPLE_MAX_BYTES  from the clique leg's 1 GiB pair (in-kernel vs
                           the event-ordered fold): the in-kernel path keeps
                           every size when it wins by the margin, else the
                           default 32 MiB stays
  NBX_LL128_ACROSS_GPUS    "1" only when the run spanned GPUs, its forced-LL128
                           stress checked >= 2000 calls with no mismatch, and
                           LL128 carries some size (DESIGN §6's flip rule)
  NBX_SIMPLE_SLICE_BYTES / NBX_SIMPLE_MAX_GRID / NBX_SIMPLE_SLOTS
                           from `collective.simple_knobs` (1 GiB AllReduce ms
                           per Simple knob setting, collective_leg.py
                           SIMPLE_KNOBS): the fastest setting when it beats the
                           default by more than the margin, else unset
Usage: python scripts/set_thresholds.py BENCH.json [--margin 0.05] [--json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from collective_leg import SIMPLE_KNOBS  # noqa: E402  (no GPU or torch import at module level)

LADDER = ("LL", "LL128", "Simple")


def last_collective_line(path: str) -> dict:
    best = None
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line.startswith("{"):
                continue
            try:
                d = json.loads(line)
            except ValueError:
                continue
            if isinstance(d.get("collective"), dict) and d["collective"].get("protocol_sweep"):
                best = d
    if best is None:
        raise SystemExit(f"{path}: no bench line with collective.protocol_sweep")
    return best


def _col(sw: dict, name: str, i: int):
    v = sw.get(name)
    return v[i] if v and i < len(v) and v[i] is not None else None


def choose(sweep: dict, n_ranks: int, margin: float = 0.05) -> dict:
    """Per swept size, the protocol carrying it under the hysteresis rule, and
    the thresholds that realise that choice."""
    sizes = sweep.get("bytes") or []
    rows = []
    cur = None
    for i, b in enumerate(sizes):
        # LL128's time at this size: the better of one-shot and the kernel the
        # library would run (two-shot above the one-shot limit when n > 2)
        t = {"LL": _col(sweep, "LL", i), "Simple": _col(sweep, "Simple", i)}
        l128 = [x for x in (_col(sweep, "LL128", i), _col(sweep, "LL128_oneshot", i)) if x is not None]
        t["LL128"] = min(l128) if l128 else None
        avail = {p: v for p, v in t.items() if v is not None}
        if not avail:
            rows.append({"bytes": b, "chosen": cur, "times_us": t})
            continue
        fastest = min(avail, key=avail.get)
        if cur is None or cur not in avail:
            # start (or the current protocol has no number here): the fastest
            # not below the current rung of the ladder
            cands = {p: v for p, v in avail.items() if cur is None or LADDER.index(p) >= LADDER.index(cur)}
            cur = min(cands, key=cands.get) if cands else fastest
        elif fastest != cur and LADDER.index(fastest) > LADDER.index(cur) and avail[cur] > avail[fastest] * (1 + margin):
            cur = fastest
        rows.append({"bytes": b, "chosen": cur, "times_us": t, "fastest": fastest})
    env = {}
    ll = [r["bytes"] for r in rows if r["chosen"] == "LL"]
    l128 = [r["bytes"] for r in rows if r["chosen"] == "LL128"]
    env["NBX_LL_MAX_BYTES"] = max(ll) if ll else 1024
    env["NBX_LL128_MAX_BYTES"] = max(l128) if l128 else 0
    if n_ranks > 2 and l128:
        one = 0
        for i, b in enumerate(sizes):
            o, t2 = _col(sweep, "LL128_oneshot", i), _col(sweep, "LL128", i)
            if o is None or t2 is None:
                continue
            if o <= t2 * (1 + margin):
                one = b
            else:
                break
        env["NBX_LL128_ONESHOT_MAX"] = one
    return {"rows": rows, "env": env}


def thresholds(bench: dict, margin: float = 0.05) -> dict:
    coll = bench["collective"]
    n = int(coll.get("n_ranks") or bench.get("n_gpus") or 2)
    out = choose(coll["protocol_sweep"], n, margin)
    env = out["env"]
    why = []
    ad, ar = (coll.get("allreduce_direct") or {}).get("ms"), (coll.get("allreduce_ring") or {}).get("ms")
    if ad and ar:
        env["NCCL_ALGO"] = "Ring" if ad > ar * (1 + margin) else ""
        why.append(f"1 GiB AllReduce: direct {ad} ms, ring {ar} ms -> "
                   f"{'ring' if env['NCCL_ALGO'] else 'direct (default)'}")
    cl = coll.get("clique") or {}
    ik, fo = cl.get("allreduce_ms"), cl.get("fold_allreduce_ms")
    if ik and fo:
        env["NBX_CLIQUE_SIMPLE_MAX_BYTES"] = (1 << 40) if fo > ik * (1 + margin) else 32 << 20
        why.append(f"clique 1 GiB AllReduce: in-kernel {ik:.4g} ms, fold {fo:.4g} ms")
    forced = coll.get("ll128_forced") or {}
    shared = bool(bench.get("shared_gpu") or coll.get("shared_gpu"))
    multi = n > 1 and not shared
    clean = forced.get("checked_calls", 0) >= 2000 and forced.get("mismatched_calls", 1) == 0
    env["NBX_LL128_ACROSS_GPUS"] = "1" if (multi and clean and env["NBX_LL128_MAX_BYTES"] > 0) else ""
    why.append(f"LL128 across GPUs: forced stress {forced.get('checked_calls')} calls, "
               f"{forced.get('mismatched_calls')} mismatched -> {'enable' if env['NBX_LL128_ACROSS_GPUS'] else 'keep off'}")
    kn = coll.get("simple_knobs") or {}
    knob_env = dict(SIMPLE_KNOBS)
    for var in sorted({v for e in knob_env.values() for v in e}):
        env[var] = ""
    base = kn.get("default")
    timed = {k: v for k, v in kn.items() if k in knob_env and v}
    if base and timed:
        best = min(timed, key=timed.get)
        if base > timed[best] * (1 + margin):
            env.update(knob_env[best])
        why.append(f"Simple knobs, 1 GiB AllReduce: default {base} ms, {timed} -> "
                   f"{best if base > timed[best] * (1 + margin) else 'default'}")
    vr = coll.get("vs_rccl") or {}
    if vr.get("sweep_best_protocol"):
        why.append(f"best protocol / RCCL per size: {vr['sweep_best_protocol']}")
    out["n_ranks"] = n
    out["margin"] = margin
    out["why"] = why
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("bench_json")
    ap.add_argument("--margin", type=float, default=0.05)
    ap.add_argument("--json", action="store_true", help="print the whole decision as JSON")
    ap.add_argument("--shared-gpu", action="store_true", help="the run's ranks shared one GPU (a rehearsal)")
    a = ap.parse_args(argv)
    b = last_collective_line(a.bench_json)
    if a.shared_gpu:
        b["shared_gpu"] = True
    res = thresholds(b, a.margin)
    if a.json:
        print(json.dumps(res, indent=1))
    else:
        for r in res["rows"]:
            print(f"# {r['bytes']:>10} B: {r['chosen']:<6} {r['times_us']}", file=sys.stderr)
        for w in res["why"]:
            print("# " + w, file=sys.stderr)
        for k, v in res["env"].items():
            print(f"export {k}={v}" if v != "" else f"unset {k}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
