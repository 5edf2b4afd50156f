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
    if d["n_wrong"]:
        s.append(f"first {d['first']} last {d['last']} runs {d['runs']}")
        s.append("explained by " + ", ".join(f"{k}={v}" for k, v in d["explained_by"].items()))
        if "cells" in d:
            s.append(f"geometry {d['geometry']}; blocks {d['blocks']}; {d['n_cells']} (block, round, workgroup) "
                     f"cells, top {d['cells']}; first at {d['first_at']} last at {d['last_at']} "
                     "(block, round, workgroup, slice offset)")
    return "; ".join(s)


def assert_same(got: np.ndarray, exp: np.ndarray, ctx, geom: SimpleGeometry | None = None, base: int = 0,
                candidates: dict | None = None) -> None:
    """Bitwise equality, or an AssertionError that says what is wrong."""
    got = np.ascontiguousarray(got)
    exp = np.ascontiguousarray(exp)
    if got.dtype != exp.dtype and got.dtype == np.uint8:
        got = got.view(exp.dtype) if got.size * got.itemsize % exp.itemsize == 0 else got
    if got.shape == exp.shape and got.dtype == exp.dtype and np.array_equal(got.view(np.uint8), exp.view(np.uint8)):
        return
    raise AssertionError(f"{ctx}: " + format_mismatch(describe_mismatch(got, exp, geom, base, candidates)))
