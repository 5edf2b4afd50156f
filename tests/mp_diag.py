"""mp_diag.py — self-describing mismatches for the multi-process collectives.

A wrong multi-process result should carry its own diagnosis (VERDICT r5,
next-round item 2): how many elements are wrong, where the first and last are,
which (block, round, workgroup, slice offset) of the Simple direct schedule
they fall in (the host's cut, comm_mp_launch.cc mpLaunchSimple /
nbx_simple.h simpleSlice), and what the wrong values look like — zero, a
peer's raw input, the fold with one source missing, the previous call's
output, ... (any candidate arrays the caller passes).

Pure numpy: the CPU suite tests the mapping with synthetic mismatches
(tests/test_mp_diag_cpu.py); the GPU tests and the stress scripts call
`assert_same` in place of a bare `np.array_equal` assert.
"""
from __future__ import annotations

import sys
from dataclasses import dataclass

import numpy as np

MIN_SLICE_BYTES = 4096   # nbx_ll_args.h kSimpleMinSliceBytes


def block_range(count: int, eb: int, n: int, b: int) -> tuple:
    """The direct schedule's block b of a count-element message: 16-B aligned
    blocks of ceil(count / n) elements rounded up to whole packs
    (nccl_api.cc blockRange)."""
    epp = 16 // eb
    per = -(-count // n)
    per = -(-per // epp) * epp
    lo = min(count, per * b)
    hi = min(count, lo + per)
    return lo, hi


@dataclass
class SimpleGeometry:
    """How one Simple launch cuts a message (comm_mp_launch.cc:114-165)."""
    kind: str           # "ar", "rs", "red" (direct schedule) or "red_ring" (ring Reduce chain)
    count: int          # elements: AllReduce / Reduce message, ReduceScatter recvcount
    eb: int             # bytes per element
    n: int
    block_elts: int
    total: int          # elements of the whole (send-side) message
    grid: int
    slice_elts: int
    n_rounds: int

    def locate(self, idx: np.ndarray) -> np.ndarray:
        """Rows (block, round, workgroup, element offset in the slice) for
        send-side element indices idx (ReduceScatter output index i of rank r
        is send-side r * count + i)."""
        idx = np.asarray(idx, dtype=np.int64)
        b = idx // self.block_elts
        off = idx - b * self.block_elts
        v = off // self.slice_elts   # virtual slice of the block: k * grid + g
        return np.stack([b, v // self.grid, v % self.grid, off - v * self.slice_elts], axis=1)


def simple_geometry(kind: str, count: int, eb: int, n: int, simple_grid: int, slice_bytes: int,
                    ring: bool = False) -> SimpleGeometry:
    """The host's cut of one single-message Simple call: block size, grid =
    min(ceil(block bytes / 4 KiB), the communicator's Simple grid), slice =
    ceil(block bytes / grid) rounded up to 16 B and capped at the staging
    slice, rounds = ceil(block bytes / (grid x slice))."""
    if kind == "rs":
        block, total = count, count * n
    elif kind == "red" and ring:
        block, total = count, count
    else:
        lo, hi = block_range(count, eb, n, 0)
        block, total = hi - lo, count
    block_bytes = min(block, total) * eb
    grid = max(1, min(-(-block_bytes // MIN_SLICE_BYTES), simple_grid))
    sl = ((-(-block_bytes // grid)) + 15) & ~15
    sl = min(sl, slice_bytes)
    rounds = -(-block_bytes // (grid * sl)) if block_bytes else 0
    return SimpleGeometry(kind, count, eb, n, max(block, 1), total, grid, max(sl // eb, 1), rounds)


def _runs(idx: np.ndarray, limit: int = 6) -> list:
    """Contiguous index runs [lo, hi) of a sorted index array (the first `limit`)."""
    if idx.size == 0:
        return []
    cut = np.nonzero(np.diff(idx) != 1)[0]
    starts = np.concatenate([[0], cut + 1])
    ends = np.concatenate([cut + 1, [idx.size]])
    return [(int(idx[s]), int(idx[e - 1]) + 1) for s, e in zip(starts[:limit], ends[:limit])]


def describe_mismatch(got: np.ndarray, exp: np.ndarray, geom: SimpleGeometry | None = None,
                      base: int = 0, candidates: dict | None = None) -> dict:
    """What is wrong in `got` (same dtype and length as `exp`).

    geom / base: the Simple cut of the call and the send-side index of got[0]
    (ReduceScatter rank r: r * recvcount), so every wrong element is mapped to
    its (block, round, workgroup, slice offset). candidates: name -> array like
    exp (or a callable idx -> values) that the wrong values are compared with —
    each candidate's count is the wrong elements it explains. Zero is always a
    candidate."""
    got = np.ascontiguousarray(got)
    exp = np.ascontiguousarray(exp)
    if got.shape != exp.shape or got.dtype != exp.dtype:
        return {"n": int(exp.size), "n_wrong": None, "shape": [list(got.shape), list(exp.shape)],
                "dtype": [str(got.dtype), str(exp.dtype)]}
    gu = got.view(np.uint8).reshape(got.size, -1) if got.size else got.view(np.uint8).reshape(0, 1)
    eu = exp.view(np.uint8).reshape(exp.size, -1) if exp.size else gu
    bad = np.nonzero((gu != eu).any(axis=1))[0]
    out = {"n": int(exp.size), "n_wrong": int(bad.size)}
    if bad.size == 0:
        return out
    out["first"], out["last"] = int(bad[0]), int(bad[-1])
    out["runs"] = _runs(bad)
    wrong = gu[bad]
    expl = {"zero": int((wrong == 0).all(axis=1).sum())}
    for name, cand in (candidates or {}).items():
        vals = cand(bad) if callable(cand) else np.ascontiguousarray(cand)[bad]
        cu = np.ascontiguousarray(vals).view(np.uint8).reshape(bad.size, -1)
        expl[name] = int((cu == wrong).all(axis=1).sum())
    out["explained_by"] = expl
    if geom is not None:
        loc = geom.locate(bad + base)
        keys, counts = np.unique(loc[:, :3], axis=0, return_counts=True)
        order = np.argsort(-counts, kind="stable")
        out["geometry"] = {"block_elts": geom.block_elts, "grid": geom.grid, "slice_elts": geom.slice_elts,
                           "rounds": geom.n_rounds}
        out["cells"] = [{"block": int(keys[i][0]), "round": int(keys[i][1]), "workgroup": int(keys[i][2]),
                         "wrong": int(counts[i])} for i in order[:8]]
        out["n_cells"] = int(len(keys))
        out["first_at"] = [int(x) for x in loc[0]]
        out["last_at"] = [int(x) for x in loc[-1]]
        out["blocks"] = {int(b): int(c) for b, c in zip(*np.unique(loc[:, 0], return_counts=True))}
    return out


def format_mismatch(d: dict) -> str:
    if d.get("n_wrong") is None:
        return f"shape/dtype differ: {d}"
    s = [f"{d['n_wrong']} of {d['n']} elements wrong"]
    if d.get("proto"):
        s[0] = f"{d['proto']}: " + s[0]
    if d["n_wrong"]:
        s.append(f"first {d['first']} last {d['last']} runs {d['runs']}")
        s.append("explained by " + ", ".join(f"{k}={v}" for k, v in d["explained_by"].items()))
        if "cells" in d:
            s.append(f"geometry {d['geometry']}; blocks {d['blocks']}; {d['n_cells']} (block, round, workgroup) "
                     f"cells, top {d['cells']}; first at {d['first_at']} last at {d['last_at']} "
                     "(block, round, workgroup, slice offset)")
    return "; ".join(s)


def compact_mismatch(d: dict) -> str:
    """One short line (<= ~160 chars) of a description: what survives a
    truncated log tail (the round-end driver keeps the last 3,000 characters)."""
    if d.get("n_wrong") is None:
        return "shape/dtype differ"
    s = f"{d.get('proto') or '?'} {d['n_wrong']}/{d['n']} wrong"
    if d["n_wrong"]:
        s += f" [{d['first']}..{d['last']}] {len(d['runs'])}{'+' if len(d['runs']) >= 8 else ''} runs"
        expl = [f"{k}={v}" for k, v in sorted(d["explained_by"].items(), key=lambda kv: -kv[1])[:3] if v]
        if expl:
            s += " = " + ",".join(expl)
        if d.get("cells"):
            c = d["cells"][0]
            s += f" cells {d['n_cells']} top b{c['block']}r{c['round']}w{c['workgroup']}:{c['wrong']}"
    return s


def emit_summary(lines) -> str:
    """Print the compact lines to stderr (pytest shows captured stderr after the
    assertion text, i.e. at the very end of the failure report) and return
    them as the message's closing block."""
    text = "SUMMARY " + " | ".join(lines)
    print(text, file=sys.stderr, flush=True)
    return text


def assert_same(got: np.ndarray, exp: np.ndarray, ctx, geom: SimpleGeometry | None = None, base: int = 0,
                candidates: dict | None = None) -> None:
    """Bitwise equality, or an AssertionError that says what is wrong."""
    got = np.ascontiguousarray(got)
    exp = np.ascontiguousarray(exp)
    if got.dtype != exp.dtype and got.dtype == np.uint8:
        got = got.view(exp.dtype) if got.size * got.itemsize % exp.itemsize == 0 else got
    if got.shape == exp.shape and got.dtype == exp.dtype and np.array_equal(got.view(np.uint8), exp.view(np.uint8)):
        return
    d = describe_mismatch(got, exp, geom, base, candidates)
    raise AssertionError(f"{ctx}: " + format_mismatch(d) + "\n" + emit_summary([f"{ctx}: {compact_mismatch(d)}"]))


def check_equal(got, exp, ctx, geom: SimpleGeometry | None = None, base: int = 0,
                candidates: dict | None = None) -> None:
    """`assert np.array_equal(got, exp), ctx` (the same pass rule), with the
    description and the compact summary when it fails."""
    got, exp = np.ascontiguousarray(got), np.ascontiguousarray(exp)
    if np.array_equal(got, exp):
        return
    if got.dtype != exp.dtype and got.shape == exp.shape:
        exp = exp.astype(got.dtype)
    d = describe_mismatch(got, exp, geom, base, candidates)
    raise AssertionError(f"{ctx}: " + format_mismatch(d) + "\n" + emit_summary([f"{ctx}: {compact_mismatch(d)}"]))


# ---------------------------------------------------------------------------
# Collective-level diagnosis (the multi-process tests and scripts/mixed_seq_repro.py)

L128_DATA_BYTES = 48   # nbx_ll_args.h kL128DataBytesHost
L128_MAX_RANKS = 8


def l128_slot_lines(max_bytes: int) -> int:
    half = (max_bytes + 1) // 2
    return 2 * (-(-half // L128_DATA_BYTES))


def proto_of(kind: str, count: int, eb: int, n: int, settings: dict, proto_mask: int = 7,
             oneshot_max: int = 256 << 10) -> str:
    """The protocol a call takes (comm_mp_init.cc chooseProtoFor), for the
    description: "LL", "LL128", "LL128x2" or "Simple"."""
    slot = count * eb
    lo, hi = block_range(count, eb, n, 0)
    block = (hi - lo) * eb
    ll_max, l128_max = settings.get("llMax", 64 << 10), settings.get("l128Max", 1 << 20)
    if slot == 0 or n > 64:
        return "Simple"
    if proto_mask & 1 and slot <= ll_max:
        return "LL"
    if proto_mask & 2 and l128_max and n <= L128_MAX_RANKS:
        if kind == "rs" or n <= 2 or slot <= oneshot_max:
            if slot <= l128_max:
                return "LL128"
        elif slot <= l128_max and block <= (l128_slot_lines(l128_max) // 2) * L128_DATA_BYTES:
            return "LL128x2"
    return "Simple"


def diagnose_collective(oracle, kind: str, dtype: int, op: int, count: int, n: int, rank: int, got_u8, xs,
                        settings: dict | None = None, prev_u8=None, root: int | None = None) -> dict:
    """Describe rank `rank`'s wrong output of one multi-process collective.

    xs: every rank's raw send buffer (oracle storage dtype, send-side length);
    kind "ar" / "rs" / "red" (Reduce: the root's output, fold order root+1,
    ..., root). Candidates: zero, each rank's raw input at the output's
    positions, the fold with one rank's source left out (per block, in the
    direct schedule's order), and `prev_u8` (this buffer position's output of
    an earlier iteration). The Simple cut is added when the call took Simple."""
    import numpy as np
    st = oracle.NP_STORAGE[dtype]
    eb = np.dtype(st).itemsize
    devop, arg = oracle.host_to_dev_redop(op, dtype, n)
    kw = dict(n_pre_op_srcs=n, post_op=devop == 4)
    if kind == "ar":
        blocks = [block_range(count, eb, n, b) for b in range(n)]
        firsts = [(b + 1) % n for b in range(n)]
        base, out_n = 0, count
    elif kind == "rs":
        blocks = [(b * count, (b + 1) * count) for b in range(n)]
        firsts = [(b + 1) % n for b in range(n)]
        base, out_n = rank * count, count
    else:
        blocks = [(0, count)]
        firsts = [((root if root is not None else 0) + 1) % n]
        base, out_n = 0, count

    def fold(skip=None):
        out = np.empty(out_n, dtype=st)
        for (lo, hi), first in zip(blocks, firsts):
            olo, ohi = max(lo - base, 0), min(hi - base, out_n)
            if ohi <= olo:
                continue
            order = [(first + k) % n for k in range(n) if (first + k) % n != skip]
            if not order:
                out[olo:ohi] = 0
                continue
            out[olo:ohi] = oracle.reduce_multi([xs[q][olo + base:ohi + base] for q in order], dtype, devop, arg,
                                               **kw)[0]
        return out

    exp = fold()
    got = np.ascontiguousarray(got_u8).view(np.uint8)[:out_n * eb].view(st)
    cand = {f"raw_input_rank{j}": np.ascontiguousarray(xs[j][base:base + out_n]) for j in range(n)}
    if n > 1:
        for j in range(n):
            cand[f"without_rank{j}"] = fold(skip=j)
    if prev_u8 is not None and np.asarray(prev_u8).size == got.size * eb:
        cand["earlier_iteration_output"] = np.ascontiguousarray(prev_u8).view(st)
    proto = proto_of(kind, count, eb, n, settings or {})
    geom = None
    if proto == "Simple" and settings:
        geom = simple_geometry(kind, count, eb, n, settings.get("simpleGrid", 32), settings.get("sliceBytes", 64 << 10),
                               ring=bool(settings.get("ring")))
    d = describe_mismatch(got, exp, geom, base, cand)
    d["proto"] = proto
    if "explained_by" in d:
        d["explained_by"] = {k: v for k, v in d["explained_by"].items() if v}
    return d


def comm_settings(nbx, comm) -> dict:
    """The communicator's transport settings (nbxDebugCommSettings) by name."""
    import ctypes
    lib = nbx.load_library()
    out = (ctypes.c_int64 * 11)()
    k = lib.nbxDebugCommSettings(comm.handle, out, 11)
    names = ["llMax", "l128Max", "sliceBytes", "slots", "simpleGrid", "llGridCap", "l128GridCap", "groupBatch",
             "ipcRepairs", "checkPlans", "checkSlices"]
    return {names[j]: int(out[j]) for j in range(max(k, 0))}


def raise_collective_failures(oracle, failures, n, what="") -> None:
    """failures: (label, kind, dtype, op, count, rank, got_u8, xs, settings, root)
    tuples; raises one AssertionError that describes up to six of them."""
    if not failures:
        return
    lines, short = [], []
    for (label, kind, dtype, op, count, rank, got, xs, settings, root) in failures[:6]:
        try:
            d = diagnose_collective(oracle, kind, dtype, op, count, n, rank, got, xs, settings, root=root)
            lines.append(f"{label} rank {rank}: {format_mismatch(d)}")
            short.append(f"{label} r{rank}: {compact_mismatch(d)}")
        except Exception as e:   # the description must never hide the failure itself
            lines.append(f"{label} rank {rank}: wrong output (diagnosis failed: {type(e).__name__}: {e})")
            short.append(f"{label} r{rank}: wrong ({type(e).__name__} in diagnosis)")
    head = f"{what}{len(failures)} wrong output(s) at {n} ranks"
    tail = emit_summary([head] + short)
    raise AssertionError(head + ":\n" + "\n".join(lines) + "\n" + tail)
