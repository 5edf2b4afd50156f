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


def _shmx_rank(name, rank, n, rounds, jitter, q):
    from tests.conftest import load_package
    nbx = load_package()
    lib = nbx.load_library()
    lib.nbxShmxSelfTest.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    q.put((rank, lib.nbxShmxSelfTest(name.encode(), rank, n, rounds, jitter)))


@pytest.mark.parametrize("n,rounds,jitter", [(1, 50, 0), (2, 400, 0), (5, 200, 200), (8, 100, 500)])
def test_shm_exchange_rounds(nbx, n, rounds, jitter):
    """The Simple path's per-call host exchange through /dev/shm: rank-stamped
    payloads of varying length, exchange numbers with gaps (LL calls in
    between skip numbers), random per-rank delays — every contribution
    verified, no rank overwriting a payload a slower peer still reads."""
    import os
    name = f"/nbx-shmx-test-{os.getpid()}-{n}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shmx_rank, args=(name, r, n, rounds, jitter, q)) for r in range(n)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=180) for _ in range(n))
        for p in procs:
            p.join(timeout=60)
    finally:
        try:
            os.unlink("/dev/shm" + name)
        except OSError:
            pass
    assert res == {r: 0 for r in range(n)}
