"""Multi-process bootstrap (the role of src/bootstrap.cc) on CPU: the unique
id from ncclGetUniqueId names a root thread in this process; N spawned
processes connect as ranks and run allgather rounds (nbxBootstrapSelfTest)."""
import ctypes
import multiprocessing as mp

import pytest


def _rank(uid_bytes, rank, n, rounds, q):
    from tests.conftest import load_package
    nbx = load_package()
    lib = nbx.load_library()
    lib.nbxBootstrapSelfTest.argtypes = [ctypes.POINTER(nbx.ncclUniqueId), ctypes.c_int, ctypes.c_int, ctypes.c_int]
    uid = nbx.ncclUniqueId.from_buffer_copy(uid_bytes)
    q.put((rank, lib.nbxBootstrapSelfTest(ctypes.byref(uid), rank, n, rounds)))


@pytest.mark.parametrize("n", [1, 2, 5])
def test_bootstrap_allgather_rounds(nbx, n):
    uid = nbx.get_unique_id()
    assert uid.internal[:8] == b"NBXUID01"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(bytes(uid), r, n, 40, q)) for r in range(n)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(n))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: 0 for r in range(n)}


def test_bootstrap_rejects_bad_args(nbx):
    lib = nbx.load_library()
    lib.nbxBootstrapSelfTest.argtypes = [ctypes.POINTER(nbx.ncclUniqueId), ctypes.c_int, ctypes.c_int, ctypes.c_int]
    uid = nbx.get_unique_id()
    assert lib.nbxBootstrapSelfTest(ctypes.byref(uid), 2, 2, 1) == 4
    assert lib.nbxBootstrapSelfTest(None, 0, 1, 1) == 4
    empty = nbx.ncclUniqueId()
    assert lib.nbxBootstrapSelfTest(ctypes.byref(empty), 0, 1, 1) == 4   # no root in the id
