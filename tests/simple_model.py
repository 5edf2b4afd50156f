"""A host model of the Simple protocol's device schedules (csrc/nbx_simple.h:
kSimpleColl, the direct schedule, and kSimpleRing) for the CPU tests.

Every (rank, workgroup) is a Python generator that runs the kernel's phases
step for step — the same slice arithmetic (simpleSlice), staging layout
(simpleStage), flag words, per-pair counters, credits and the next-round
prefetch — yielding whenever the kernel would spin on a flag. A scheduler
interleaves them (round robin or seeded random order) until every one has
finished, or reports a deadlock if none can move. Data moves through numpy
byte arrays, folds through the oracle's ordered left fold. Test
infrastructure only (nothing in the product imports it)."""
from __future__ import annotations

import random

import numpy as np

RS_READY, RS_CREDIT, AG_READY, AG_CREDIT = 0, 1, 2, 3      # flag kinds (nbx_ll_args.h SimpleFlag)
RS_SENT, RS_RECV, AG_SENT, AG_RECV = 0, 1, 2, 3            # counters (SimpleCounter)
MIN_SLICE = 4096                                           # kSimpleMinSliceBytes


class Comm:
    """The init-time state of one multi-process communicator (all ranks)."""

    def __init__(self, n, grid_max, slice_bytes, slots):
        self.n, self.gm, self.slice, self.slots = n, grid_max, slice_bytes, slots
        cells = n * grid_max
        self.stage = [np.zeros(2 * slots * cells * slice_bytes, np.uint8) for _ in range(n)]
        self.flags = [np.zeros(4 * cells, np.uint64) for _ in range(n)]
        self.counters = [np.zeros(4 * cells, np.uint64) for _ in range(n)]

    def stage_off(self, region, slot, src, g):
        return ((((region * self.slots + slot) * self.n + src) * self.gm) + g) * self.slice

    def flag_idx(self, kind, who, g):
        return (kind * self.n + who) * self.gm + g


def call_shape(comm, kind, count, eb, ring):
    """mpLaunchSimple: (blockElts, total, grid, slice, rounds)."""
    n = comm.n
    if kind == "rs":
        block, total = count, count * n
    elif kind == "red" and ring:
        block, total = count, count
    else:
        epp = 16 // eb
        per = -(-count // n)
        block, total = -(-per // epp) * epp, count
    bb = min(block, total) * eb
    if bb == 0:
        return None
    grid = max(1, min(-(-bb // MIN_SLICE), comm.gm))
    sl = min((-(-bb // grid) + 15) // 16 * 16, comm.slice)
    rounds = -(-bb // (grid * sl))
    return block, total, grid, sl, rounds


def _slice(block, total, sl_elts, grid, b, k, g):
    lo = min(b * block, total)
    hi = total if total - lo < block else lo + block
    s0 = (k * grid + g) * sl_elts
    return lo + s0, (0 if s0 >= hi - lo else min(hi - lo - s0, sl_elts))


def _wg(comm, me, g, kind, ring, shape, send, recv, eb, fold, root, prefetch, stats):
    """One workgroup of one rank's kernel (a generator; yields while spinning)."""
    n, slots = comm.n, comm.slots
    block, total, grid, sl, rounds = shape
    sle = sl // eb
    cnt = {c: [int(comm.counters[me][comm.flag_idx(c, p, g)]) for p in range(n)] for c in range(4)}
    my_flags = comm.flags[me]

    def flag(kind_, who):
        return int(my_flags[comm.flag_idx(kind_, who, g)])

    def post(to, kind_, value):
        comm.flags[to][comm.flag_idx(kind_, me, g)] = value

    def wait(kind_, who, target):
        while flag(kind_, who) < target:
            stats["spins"] += 1
            yield
        stats["moves"] += 1

    def stage(owner, region, slot, src, nbytes):
        o = comm.stage_off(region, slot, src, g)
        assert nbytes <= comm.slice, "slice larger than a staging slot"
        return comm.stage[owner][o:o + nbytes]

    def elts(buf, off, c):
        return buf[off * eb:(off + c) * eb]

    if not ring:
        ar, red = kind == "ar", kind == "red"
        store_local = not red or me == root
        gathers = ar or (red and me == root)
        first = ((root if red else me) + 1) % n

        def push_target(p):
            return p != me and (ar or (red and p == root))

        def phase_a(k):
            for t in range(n):
                if t != me and cnt[RS_SENT][t] + 1 > slots:
                    yield from wait(RS_CREDIT, t, cnt[RS_SENT][t] + 1 - slots)
            for q in range(1, n):
                j = (me + q) % n
                off, c = _slice(block, total, sle, grid, j, k, g)
                if c:
                    stage(j, 0, cnt[RS_SENT][j] % slots, me, c * eb)[:] = elts(send, off, c)
            for t in range(n):
                if t != me:
                    cnt[RS_SENT][t] += 1
                    post(t, RS_READY, cnt[RS_SENT][t])

        def phase_b(k):
            for t in range(n):
                if t != me:
                    yield from wait(RS_READY, t, cnt[RS_RECV][t] + 1)
                    if push_target(t) and cnt[AG_SENT][t] + 1 > slots:
                        yield from wait(AG_CREDIT, t, cnt[AG_SENT][t] + 1 - slots)
            off, c = _slice(block, total, sle, grid, me, k, g)
            if c:
                srcs = []
                for q in range(n):
                    j = (first + q) % n
                    srcs.append(elts(send, off, c) if j == me else stage(me, 0, cnt[RS_RECV][j] % slots, j, c * eb))
                res = fold(srcs)
                if store_local:
                    elts(recv, off - me * block if kind == "rs" else off, c)[:] = res
                for q in range(1, n):
                    p = (me + q) % n
                    if push_target(p):
                        stage(p, 1, cnt[AG_SENT][p] % slots, me, c * eb)[:] = res
            for t in range(n):
                if t != me:
                    cnt[RS_RECV][t] += 1
                    post(t, RS_CREDIT, cnt[RS_RECV][t])
                    if push_target(t):
                        cnt[AG_SENT][t] += 1
                        post(t, AG_READY, cnt[AG_SENT][t])

        def phase_c(k):
            for t in range(n):
                if t != me:
                    yield from wait(AG_READY, t, cnt[AG_RECV][t] + 1)
            for q in range(1, n):
                j = (me + q) % n
                off, c = _slice(block, total, sle, grid, j, k, g)
                if c:
                    elts(recv, off, c)[:] = stage(me, 1, cnt[AG_RECV][j] % slots, j, c * eb)
            for t in range(n):
                if t != me:
                    cnt[AG_RECV][t] += 1
                    post(t, AG_CREDIT, cnt[AG_RECV][t])

        if prefetch and rounds > 0:
            yield from phase_a(0)
        for k in range(rounds):
            if prefetch:
                if k + 1 < rounds:
                    yield from phase_a(k + 1)
            else:
                yield from phase_a(k)
            yield from phase_b(k)
            if gathers:
                yield from phase_c(k)
    else:
        left, right = (me + n - 1) % n, (me + 1) % n
        ar, red = kind == "ar", kind == "red"

        def hop_wait(recv_region, push_rs, push_ag):
            if recv_region >= 0:
                yield from wait(RS_READY if recv_region == 0 else AG_READY, left,
                                cnt[RS_RECV if recv_region == 0 else AG_RECV][left] + 1)
            if push_rs and cnt[RS_SENT][right] + 1 > slots:
                yield from wait(RS_CREDIT, right, cnt[RS_SENT][right] + 1 - slots)
            if push_ag and cnt[AG_SENT][right] + 1 > slots:
                yield from wait(AG_CREDIT, right, cnt[AG_SENT][right] + 1 - slots)

        def hop_post(recv_region, push_rs, push_ag):
            if recv_region == 0:
                cnt[RS_RECV][left] += 1
                post(left, RS_CREDIT, cnt[RS_RECV][left])
            if recv_region == 1:
                cnt[AG_RECV][left] += 1
                post(left, AG_CREDIT, cnt[AG_RECV][left])
            if push_rs:
                cnt[RS_SENT][right] += 1
                post(right, RS_READY, cnt[RS_SENT][right])
            if push_ag:
                cnt[AG_SENT][right] += 1
                post(right, AG_READY, cnt[AG_SENT][right])

        for k in range(rounds):
            if red:
                pos = (me - root - 1 + 2 * n) % n
                off, c = _slice(block, total, sle, grid, 0, k, g)
                push = pos < n - 1
                yield from hop_wait(-1 if pos == 0 else 0, push, False)
                if c:
                    if pos == 0:
                        out = elts(send, off, c)
                    else:
                        recv_part = stage(me, 0, cnt[RS_RECV][left] % slots, left, c * eb)
                        out = fold([elts(send, off, c), recv_part], pre_mask=3 if pos == 1 else 1, post=not push)
                    if push:
                        stage(right, 0, cnt[RS_SENT][right] % slots, me, c * eb)[:] = out
                    else:
                        elts(recv, off, c)[:] = out
                hop_post(-1 if pos == 0 else 0, push, False)
                continue
            off, c = _slice(block, total, sle, grid, left, k, g)
            yield from hop_wait(-1, True, False)
            if c:
                stage(right, 0, cnt[RS_SENT][right] % slots, me, c * eb)[:] = elts(send, off, c)
            hop_post(-1, True, False)
            for st in range(n - 1):
                ch = (me + 2 * n - 2 - st) % n
                last = st == n - 2
                off, c = _slice(block, total, sle, grid, ch, k, g)
                yield from hop_wait(0, not last, last and ar)
                if c:
                    recv_part = stage(me, 0, cnt[RS_RECV][left] % slots, left, c * eb)
                    out = fold([elts(send, off, c), recv_part], pre_mask=3 if st == 0 else 1, post=last)
                    if last:
                        elts(recv, off if ar else off - me * block, c)[:] = out
                        if ar:
                            stage(right, 1, cnt[AG_SENT][right] % slots, me, c * eb)[:] = out
                    else:
                        stage(right, 0, cnt[RS_SENT][right] % slots, me, c * eb)[:] = out
                hop_post(0, not last, last and ar)
            if not ar:
                continue
            for st in range(n - 1):
                ch = (me + 2 * n - 1 - st) % n
                fwd = st < n - 2
                off, c = _slice(block, total, sle, grid, ch, k, g)
                yield from hop_wait(1, False, fwd)
                if c:
                    part = stage(me, 1, cnt[AG_RECV][left] % slots, left, c * eb)
                    elts(recv, off, c)[:] = part
                    if fwd:
                        stage(right, 1, cnt[AG_SENT][right] % slots, me, c * eb)[:] = part
                hop_post(1, False, fwd)
    for c_ in range(4):
        for p in range(n):
            comm.counters[me][comm.flag_idx(c_, p, g)] = cnt[c_][p]


def run_call(comm, kind, sends, recvs, count, eb, fold, root=0, ring=False, prefetch=True, order="rr", seed=0,
             max_steps=10_000_000):
    """Run one collective on every rank; sends / recvs are per-rank uint8 arrays
    (recv None on Reduce non-roots). fold(srcs, pre_mask=..., post=...) folds
    byte arrays of one dtype. Returns the scheduler statistics."""
    shape = call_shape(comm, kind, count, eb, ring)
    stats = {"spins": 0, "steps": 0, "moves": 0}
    if shape is None:
        return stats
    gens = []
    for r in range(comm.n):
        for g in range(shape[2]):
            gens.append(_wg(comm, r, g, kind, ring, shape, sends[r], recvs[r], eb,
                            fold, root, prefetch, stats))
    rng = random.Random(seed)
    live = list(gens)
    stuck = 0
    while live:
        stats["steps"] += 1
        assert stats["steps"] < max_steps, "simulation did not finish"
        if order == "random":
            rng.shuffle(live)
        progressed = False
        nxt = []
        for gen in live:
            before = stats["moves"]
            try:
                next(gen)
                nxt.append(gen)
                progressed |= stats["moves"] != before
            except StopIteration:
                progressed = True
        live = nxt
        stuck = 0 if progressed else stuck + 1
        assert stuck < 3, f"deadlock: {len(live)} workgroups spinning"
    return stats
