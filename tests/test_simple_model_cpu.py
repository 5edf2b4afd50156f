"""CPU model of the Simple protocol's device schedules (tests/simple_model.py
restates csrc/nbx_simple.h step for step): every output exact, no deadlock,
counters consistent across many calls of varying shape on one communicator —
with workgroups interleaved round robin and in seeded random order, with and
without the next-round prefetch, direct and ring schedules."""
import numpy as np
import pytest

from tests import simple_model as sm


def _fold(srcs, pre_mask=None, post=True):
    acc = srcs[0].view(np.float32).astype(np.float64)
    for s in srcs[1:]:
        acc = acc + s.view(np.float32)
    return acc.astype(np.float32).view(np.uint8)


def _run(n, ring, prefetch, order, calls, grid_max=4, slice_bytes=4096, slots=2, seed=0):
    comm = sm.Comm(n, grid_max, slice_bytes, slots)
    rng = np.random.default_rng(seed)
    for ci, (kind, count) in enumerate(calls):
        root = ci % n
        total = count * n if kind == "rs" else count
        xs = [rng.integers(0, 100, total).astype(np.float32) for _ in range(n)]
        out_n = count
        recvs = [np.full(out_n, -1, np.float32).view(np.uint8).copy() if (kind != "red" or r == root) else None
                 for r in range(n)]
        sends = [x.view(np.uint8).copy() for x in xs]
        sm.run_call(comm, kind, sends, recvs, count, 4, _fold, root=root, ring=ring, prefetch=prefetch,
                    order=order, seed=seed + ci)
        full = np.sum(xs, axis=0).astype(np.float32)
        for r in range(n):
            if recvs[r] is None:
                continue
            got = recvs[r].view(np.float32)
            want = full[r * count:(r + 1) * count] if kind == "rs" else full
            assert np.array_equal(got, want), (kind, count, r, ring, prefetch, order,
                                               int((got != want).sum()))


CALLS = [("ar", 1), ("ar", 1000), ("ar", 4099), ("rs", 777), ("red", 5000), ("ar", 40009), ("rs", 1024),
         ("red", 3), ("ar", 16384 * 3 + 5)]


@pytest.mark.parametrize("n", [2, 3, 5])
@pytest.mark.parametrize("ring", [False, True])
@pytest.mark.parametrize("prefetch", [False, True])
@pytest.mark.parametrize("order", ["rr", "random"])
def test_simple_protocol_model(n, ring, prefetch, order):
    _run(n, ring, prefetch, order, CALLS, seed=n * 7 + ring * 3 + prefetch)


@pytest.mark.parametrize("n,slots,grid_max,slice_bytes", [(8, 2, 3, 4096), (9, 3, 2, 8192), (4, 4, 5, 4096)])
@pytest.mark.parametrize("ring", [False, True])
def test_simple_protocol_model_shapes(n, slots, grid_max, slice_bytes, ring):
    """More ranks than the 8-source reduce kernels, deeper slot rings, grids
    that do not divide the blocks, several rounds per call."""
    calls = [("ar", 100003), ("rs", 5003), ("red", 70001), ("ar", 7), ("rs", 1), ("ar", 64 * 1024)]
    _run(n, ring, True, "random", calls, grid_max=grid_max, slice_bytes=slice_bytes, slots=slots, seed=n + slots)
