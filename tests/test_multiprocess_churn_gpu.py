"""Multi-process communicators under the allocation churn real callers have
(VERDICT r2 items 1-2): between collectives, tensors are freed and
re-allocated at varying sizes, torch.cuda.empty_cache() returns segments to
the driver, and communicators are created and destroyed in sequence.

The first case reproduces the round-2 bench rehearsal's failing sequence
deterministically: 2 ranks; large buffers used by a communicator, freed,
empty_cache, the communicator destroyed; a NEW communicator; its first Simple
1 MiB AllReduce into a -1 sentinel. In round 2 rank 1's view of rank 0's new
buffer read stale bytes and its stores never landed (profiles/r2/rehearsal_r4z.jsonl).

Inputs are small integers in fp32 / int32, so every fold order gives the exact
result and the expected output is computed independently of the library (the
reference's Sum on such values is exact; reduce_kernel.h:147-150). Every
output starts as a -1 sentinel, so an element nobody wrote is caught.
All ranks share the test box's one GPU."""
import multiprocessing as mp

import pytest

pytestmark = pytest.mark.gpu

BIG = 64 << 20            # bytes per rank for the large phase-1 buffers
FIRST = 1 << 20           # the rehearsal's failing message: 1 MiB fp32
SIZES = [4 << 10, 96 << 10, 1 << 20, 3 << 20, (5 << 20) + 12, 24 << 20]
CHURN_ITERS = 14


def _vals(torch, n_elts, r, salt, dtype):
    idx = torch.arange(n_elts, dtype=torch.int64, device="cuda")
    return ((idx * 5 + 3 * r + salt) % 509).to(dtype)


def _expect(torch, n_elts, world, salt, dtype):
    idx = torch.arange(n_elts, dtype=torch.int64, device="cuda")
    acc = torch.zeros(n_elts, dtype=torch.int64, device="cuda")
    for r in range(world):
        acc += (idx * 5 + 3 * r + salt) % 509
    return acc.to(dtype)


def _describe(torch, got, want, own):
    bad = (got != want).nonzero().flatten()
    i0, i1 = int(bad[0]), int(bad[-1])
    return (f"{bad.numel()} of {got.numel()} elements differ in [{i0}, {i1}] (got {got[i0].item()} want "
            f"{want[i0].item()}; unwritten {int((got[bad] == -1).sum())}, equal to own input "
            f"{int((got[bad] == own[bad]).sum()) if own is not None else 'n/a'})")


def _child(uids, rank, n, q, algo):
    try:
        import os
        import random
        os.environ["NCCL_PROTO"] = "" if algo == "default" else "Simple"
        os.environ["NCCL_ALGO"] = "Ring" if algo == "ring" else ""
        import torch
        from tests.conftest import load_package
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        st = torch.cuda.current_stream().cuda_stream
        errors = []
        F32, I32, SUM, MAX = 7, 2, 0, 2

        def init(k):
            return nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uids[k]), rank)

        def all_reduce(comm, nbytes, salt, dtype=torch.float32, code=F32, tag=""):
            cnt = nbytes // 4
            x = _vals(torch, cnt, rank, salt, dtype)
            y = torch.full((cnt,), -1, dtype=dtype, device="cuda")
            comm.all_reduce(x.data_ptr(), y.data_ptr(), cnt, code, SUM, st)
            torch.cuda.synchronize()
            want = _expect(torch, cnt, n, salt, dtype)
            if not torch.equal(y, want):
                errors.append(f"{tag} allreduce {nbytes} B: " + _describe(torch, y, want, x))

        # phase 1: a communicator moves large buffers, which are then freed and
        # returned to the driver (empty_cache), and the communicator destroyed
        comm_a = init(0)
        all_reduce(comm_a, BIG, 1, tag="phase1")
        all_reduce(comm_a, BIG // 2, 2, tag="phase1")
        torch.cuda.empty_cache()
        comm_a.destroy()
        # phase 2: a NEW communicator's first Simple 1 MiB AllReduce (the r2 failure)
        comm = init(1)
        all_reduce(comm, FIRST, 3, tag="first-call")
        # phase 3: churn — fresh tensors of varying sizes every call, empty_cache
        # and unrelated per-rank allocations in between
        rng = random.Random(99)              # identical call sequence on every rank
        junk_rng = random.Random(7 + rank)   # per-rank allocator noise
        junk = []
        for it in range(CHURN_ITERS):
            nbytes = rng.choice(SIZES)
            kind = rng.choice(["ar", "ar", "rs", "red", "ar_i32_max"])
            if junk_rng.random() < 0.5:
                junk.append(torch.empty(junk_rng.choice([1 << 20, 20 << 20, 200 << 20]), dtype=torch.uint8,
                                        device="cuda"))
            if junk and junk_rng.random() < 0.5:
                junk.pop(junk_rng.randrange(len(junk)))
            if rng.random() < 0.5:
                torch.cuda.empty_cache()
            salt = 10 + it
            if kind == "ar":
                all_reduce(comm, nbytes, salt, tag=f"churn{it}")
            elif kind == "ar_i32_max":
                cnt = nbytes // 4
                x = _vals(torch, cnt, rank, salt, torch.int32)
                y = torch.full((cnt,), -1, dtype=torch.int32, device="cuda")
                comm.all_reduce(x.data_ptr(), y.data_ptr(), cnt, I32, MAX, st)
                torch.cuda.synchronize()
                idx = torch.arange(cnt, dtype=torch.int64, device="cuda")
                want = torch.stack([(idx * 5 + 3 * r + salt) % 509 for r in range(n)]).max(0).values.to(torch.int32)
                if not torch.equal(y, want):
                    errors.append(f"churn{it} allreduce int32 max {nbytes} B: " + _describe(torch, y, want, x))
            elif kind == "rs":
                rc = max(4, nbytes // 4 // n)
                x = _vals(torch, rc * n, rank, salt, torch.float32)
                y = torch.full((rc,), -1.0, device="cuda")
                comm.reduce_scatter(x.data_ptr(), y.data_ptr(), rc, F32, SUM, st)
                torch.cuda.synchronize()
                want = _expect(torch, rc * n, n, salt, torch.float32)[rank * rc:(rank + 1) * rc]
                if not torch.equal(y, want):
                    errors.append(f"churn{it} reducescatter {rc} elts: " + _describe(torch, y, want, None))
            else:
                cnt = nbytes // 4
                root = it % n
                x = _vals(torch, cnt, rank, salt, torch.float32)
                y = torch.full((cnt,), -1.0, device="cuda")
                comm.reduce(x.data_ptr(), y.data_ptr() if rank == root else 0, cnt, F32, SUM, root, st)
                torch.cuda.synchronize()
                if rank == root:
                    want = _expect(torch, cnt, n, salt, torch.float32)
                    if not torch.equal(y, want):
                        errors.append(f"churn{it} reduce {nbytes} B root {root}: " + _describe(torch, y, want, x))
        del junk
        if comm.async_error() != 0:
            errors.append("async error")
        comm.destroy()
        # phase 4: communicators created and destroyed in sequence
        for k in range(3):
            torch.cuda.empty_cache()
            c = init(2 + k)
            all_reduce(c, (k + 1) << 20, 40 + k, tag=f"comm{k}")
            c.destroy()
        q.put((rank, "ok", errors))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("n,algo", [(2, "direct"), (2, "ring"), (3, "direct"), (3, "ring"), (3, "default"),
                                    (8, "direct")])
def test_multiprocess_allocation_churn(nbx, n, algo, monkeypatch):
    """Every output exact under free / re-allocate / empty_cache and
    communicator create / destroy churn (Simple protocol forced except
    `default`; `ring` = NCCL_ALGO=Ring)."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NBX_LL128_MAX_GRID", "16")
    monkeypatch.setenv("NBX_LL_MAX_GRID", "32")
    monkeypatch.setenv("NBX_SIMPLE_MAX_GRID", "16")
    uids = [bytes(nbx.get_unique_id()) for _ in range(5)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_child, args=(uids, r, n, q, algo), daemon=True) for r in range(n)]
    for p in procs:
        p.start()
    errs = {}
    try:
        for _ in range(n):
            rank, status, payload = q.get(timeout=300)
            assert status == "ok", f"rank {rank}:\n{payload}"
            errs[rank] = payload
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
    bad = {r: e for r, e in errs.items() if e}
    assert not bad, bad
