"""Multi-process communicators (one process per rank, ncclCommInitRank with
nranks > 1) on the GPU box. The box has one GPU, so the ranks share device 0:
this exercises the bootstrap, the connection buffers every peer IPC-maps once
at init, and the LL / LL128 / Simple (direct and ring) kernels with their
in-kernel flow control end to end. Results are compared bit-exact with the
oracle folding block r in rank order r+1, ..., r."""
import multiprocessing as mp

import numpy as np
import pytest

from tests import mp_diag

pytestmark = pytest.mark.gpu

CASES = [  # (kind, dtype, op)
    ("allreduce", 7, 0), ("allreduce", 7, 4), ("allreduce", 6, 0), ("allreduce", 2, 4), ("allreduce", 4, 2),
    ("reducescatter", 7, 0), ("reducescatter", 9, 4), ("reduce", 7, 0), ("reduce", 2, 4),
]
COUNT = 40009


def _inputs(oracle, kind, dtype, n, r):
    cnt = COUNT * n if kind == "reducescatter" else COUNT
    return oracle.random_inputs(dtype, n, cnt, seed=1000 + 10 * dtype)[r]


def _child(uid_bytes, rank, n, q, grouped=False):
    """grouped: every round's CASES go into ONE ncclGroupStart/End (the
    multi-process group batching: queued, exchanged, run as batched
    exchanges), plus an AllReduce that reads the first case's output (a
    dependency that must split the batch), with every buffer alive until the
    group ends."""
    try:
        import torch
        from tests.conftest import load_package
        from oracle import oracle
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        uid = nbx.ncclUniqueId.from_buffer_copy(uid_bytes)
        comm = nbx.Communicator.init_rank(n, uid, rank)
        assert comm.count() == n and comm.user_rank() == rank
        st = torch.cuda.Stream()
        out = {"settings": mp_diag.comm_settings(nbx, comm)}
        if grouped:
            for it in range(2):
                live = []
                nbx.group_start()
                for kind, dtype, op in CASES:
                    x = _inputs(oracle, kind, dtype, n, rank)
                    tx = torch.from_numpy(x.view(np.uint8).copy()).cuda()
                    nbytes = (COUNT if kind == "reducescatter" else x.size) * x.itemsize
                    ty = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
                    torch.cuda.synchronize()
                    if kind == "allreduce":
                        comm.all_reduce(tx.data_ptr(), ty.data_ptr(), x.size, dtype, op, st.cuda_stream)
                    elif kind == "reducescatter":
                        comm.reduce_scatter(tx.data_ptr(), ty.data_ptr(), COUNT, dtype, op, st.cuda_stream)
                    else:
                        comm.reduce(tx.data_ptr(), ty.data_ptr() if rank == 1 % n else 0, x.size, dtype, op,
                                    1 % n, st.cuda_stream)
                    live.append((kind, dtype, op, tx, ty))
                first_out = live[0][4]   # ("allreduce", 7, 0)
                dep = torch.zeros_like(first_out)
                comm.all_reduce(first_out.data_ptr(), dep.data_ptr(), COUNT, 7, 0, st.cuda_stream)
                # right behind it, same kind / type / op / size: a run candidate
                # that reads what the call before it writes (must be cut there)
                dep2 = torch.zeros_like(first_out)
                comm.all_reduce(dep.data_ptr(), dep2.data_ptr(), COUNT, 7, 0, st.cuda_stream)
                nbx.group_end()
                st.synchronize()
                for kind, dtype, op, tx, ty in live:
                    out[(it, kind, dtype, op)] = ty.cpu().numpy().copy()
                out[(it, "dep")] = dep.cpu().numpy().copy()
                out[(it, "dep2")] = dep2.cpu().numpy().copy()
        for it in range(0 if grouped else 2):   # twice: the second round hits the IPC mapping cache
            for kind, dtype, op in CASES:
                x = _inputs(oracle, kind, dtype, n, rank)
                tx = torch.from_numpy(x.view(np.uint8).copy()).cuda()
                nbytes = (COUNT if kind == "reducescatter" else x.size) * x.itemsize
                ty = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                if kind == "allreduce":
                    comm.all_reduce(tx.data_ptr(), ty.data_ptr(), x.size, dtype, op, st.cuda_stream)
                elif kind == "reducescatter":
                    comm.reduce_scatter(tx.data_ptr(), ty.data_ptr(), COUNT, dtype, op, st.cuda_stream)
                else:
                    comm.reduce(tx.data_ptr(), ty.data_ptr() if rank == 1 % n else 0, x.size, dtype, op, 1 % n,
                                st.cuda_stream)
                st.synchronize()
                out[(it, kind, dtype, op)] = ty.cpu().numpy().copy()
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", out))
    except Exception as e:  # report, never hang the parent
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def _blocks(count, eb, n):
    epp = 16 // eb
    per = -(-count // n)
    per = -(-per // epp) * epp
    return [(min(count, per * b), min(count, per * b + per)) for b in range(n)]


@pytest.mark.parametrize("n,algo,proto,slice_", [(2, "direct", "LL,Simple", ""), (3, "direct", "LL,Simple", ""),
                                                 (3, "ring", "LL,Simple", ""), (4, "ring", "LL,Simple", ""),
                                                 (5, "ring", "LL,Simple", ""), (4, "direct", "LL,Simple", "4096"),
                                                 (3, "direct", "", ""), (9, "direct", "LL,Simple", "")])
def test_multiprocess_collectives(nbx, oracle, n, algo, proto, slice_, monkeypatch):
    """NCCL_ALGO=Ring: NCCL's ring order (chunk c from rank c+1 to c, Fn(local,
    received)); for the commutative ops tested it is bit-identical to the
    oracle's left fold in the order c+1, ..., c. NCCL_PROTO=LL,Simple keeps the
    40009-element messages on the Simple (direct / ring) path; the default
    sends most of them through LL128. NBX_SIMPLE_SLICE_BYTES=4096 with a grid of
    2 makes every call run many rounds through the 2 staging slots; 9 ranks:
    more sources than the 8-source reduce kernels (the fold runs in groups)."""
    # bounded waits everywhere: a failing rank must not strand its peers
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NBX_LL128_MAX_GRID", "16")
    monkeypatch.setenv("NCCL_PROTO", proto)
    monkeypatch.setenv("NCCL_ALGO", "Ring" if algo == "ring" else "")
    monkeypatch.setenv("NBX_SIMPLE_SLICE_BYTES", slice_)
    monkeypatch.setenv("NBX_SIMPLE_MAX_GRID", "2" if slice_ else "")
    res = _run_ranks(nbx, n, _child)
    _check_cases(oracle, n, res)


@pytest.mark.parametrize("n,proto", [(2, "LL,Simple"), (3, "LL,Simple"), (3, ""), (9, "LL,Simple")])
def test_multiprocess_grouped_collectives(nbx, oracle, n, proto, monkeypatch):
    """One ncclGroupStart/End around every case: the calls are queued and run
    at ncclGroupEnd — independent Simple calls as one batched exchange, LL /
    LL128 calls in order, the dependent AllReduce after the call it reads.
    Results are the same as one call at a time (bit-exact); 9 ranks: AllReduce
    needs the gather step there and runs alone."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NBX_LL128_MAX_GRID", "16")
    monkeypatch.setenv("NBX_LL_MAX_GRID", "64")
    monkeypatch.setenv("NCCL_PROTO", proto)
    monkeypatch.setenv("NCCL_ALGO", "")
    res = _run_ranks(nbx, n, _child, True)
    _check_cases(oracle, n, res)
    # the dependent AllReduce summed n copies of case ("allreduce", 7, 0)'s result
    first = [res[r][(0, "allreduce", 7, 0)].view(np.float32) for r in range(n)]
    blocks = _blocks(COUNT, 4, n)
    exp = np.empty(COUNT, dtype=np.float32)
    for r, (lo, hi) in enumerate(blocks):
        if hi > lo:
            order = [(r + 1 + k) % n for k in range(n)]
            exp[lo:hi] = oracle.reduce_multi([first[j][lo:hi] for j in order], 7, 0, 0, n_pre_op_srcs=n)[0]
    exp2 = np.empty(COUNT, dtype=np.float32)
    for r, (lo, hi) in enumerate(blocks):
        if hi > lo:
            exp2[lo:hi] = oracle.reduce_multi([exp[lo:hi]] * n, 7, 0, 0, n_pre_op_srcs=n)[0]
    for it in range(2):
        for r in range(n):
            mp_diag.check_equal(res[r][(it, "dep")].view(np.float32), exp, ("dep", it, r))
            mp_diag.check_equal(res[r][(it, "dep2")].view(np.float32), exp2, ("dep2", it, r))


def _run_ranks(nbx, n, target, *extra):
    uid = nbx.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(bytes(uid), r, n, q, *extra), daemon=True) for r in range(n)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(n):
            rank, status, payload = q.get(timeout=300)
            assert status == "ok", f"rank {rank}:\n{payload}"
            res[rank] = payload
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
    return res


def _check_cases(oracle, n, res):
    failures = []
    for kind, dtype, op in CASES:
        xs = [_inputs(oracle, kind, dtype, n, r) for r in range(n)]
        devop, arg = oracle.host_to_dev_redop(op, dtype, n)
        st = oracle.NP_STORAGE[dtype]
        eb = np.dtype(st).itemsize
        if kind == "reducescatter":
            blocks = [(b * COUNT, (b + 1) * COUNT) for b in range(n)]
        else:
            blocks = _blocks(xs[0].size, eb, n)
        full = np.empty(xs[0].size, dtype=st)
        for r, (lo, hi) in enumerate(blocks):
            if hi > lo:
                first = (1 % n if kind == "reduce" else r) + 1   # Reduce: chain order toward root 1 % n
                order = [(first + k) % n for k in range(n)]
                full[lo:hi] = oracle.reduce_multi([xs[j][lo:hi] for j in order], dtype, devop, arg,
                                                  n_pre_op_srcs=n, post_op=devop == 4)[0]
        for it in range(2):
            for r in range(n):
                got = res[r][(it, kind, dtype, op)].view(st)
                if kind == "allreduce":
                    exp = full
                elif kind == "reducescatter":
                    exp = full[r * COUNT:(r + 1) * COUNT]
                else:
                    if r != 1 % n:
                        continue
                    exp = full
                if not np.array_equal(got.view(np.uint8), exp.view(np.uint8)):
                    k = {"allreduce": "ar", "reducescatter": "rs", "reduce": "red"}[kind]
                    failures.append((f"iteration {it} {kind} dtype {dtype} op {op}", k, dtype, op, COUNT, r,
                                     got.view(np.uint8), xs, res[r].get("settings"), 1 % n))
    mp_diag.raise_collective_failures(oracle, failures, n)


# NCCL_ALGO=Ring ReduceScatter / Reduce through the Simple ring schedule
# (nbx_simple.h kSimpleRing, hop for hop through the right neighbour's
# staging): (kind, dtype, op, count, root). Blocks that are not whole 16-B
# packs (the bf16 RS of 777) take the element path; Reduce counts with a
# partial last pack exercise the element tail.
RING_FIFO_CASES = [
    ("rs", 7, 0, 4096, 0), ("rs", 6, 4, 1 << 20, 0), ("rs", 2, 2, 300000, 0), ("rs", 9, 0, 777, 0),
    ("rs", 8, 1, 65536, 0), ("red", 7, 0, 1000003, 0), ("red", 7, 0, 250000, -1), ("red", 8, 1, 200001, 1),
    ("red", 0, 0, 123457, 1), ("red", 6, 4, 99999, -1),
]


def _ring_fifo_input(kind, dtype, count, n, r):
    from oracle import oracle
    total = count * n if kind == "rs" else count
    return oracle.random_inputs(dtype, 8, total, seed=500 + dtype + count % 1000)[r]


def _child_ring_fifo(uid_bytes, rank, n, q):
    try:
        import torch
        from tests.conftest import load_package
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        st = torch.cuda.current_stream().cuda_stream
        out = {}
        for it in range(2):   # twice: cumulative FIFO counts carry across calls
            for i, (kind, dtype, op, count, root) in enumerate(RING_FIFO_CASES):
                root = root % n
                x = _ring_fifo_input(kind, dtype, count, n, rank)
                tx = torch.from_numpy(x.view(np.uint8).copy()).cuda()
                nb = (count * x.itemsize) if kind == "rs" else x.nbytes
                ty = torch.zeros(nb, dtype=torch.uint8, device="cuda")
                if kind == "rs":
                    comm.reduce_scatter(tx.data_ptr(), ty.data_ptr(), count, dtype, op, st)
                else:
                    comm.reduce(tx.data_ptr(), ty.data_ptr() if rank == root else 0, count, dtype, op, root, st)
                torch.cuda.synchronize()
                out[(it, i)] = ty.cpu().numpy().copy()
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def ring_chain(oracle, parts, dtype, devop, arg, n):
    """NCCL's ring / chain accumulation, operand for operand: the first hop
    folds Fn(pre(x1), pre(x0)) (local input, the left neighbour's raw input),
    every later hop Fn(pre(local), received), postOp on the last
    (reduce_scatter.h:49-64, reduce.h:44-67, prims_simple.h genericOp)."""
    if n == 1:
        return oracle.reduce_multi([parts[0]], dtype, devop, arg, n_pre_op_srcs=1, post_op=devop == 4)[0]
    acc = None
    for k in range(1, n):
        last = k == n - 1
        if k == 1:
            acc = oracle.reduce_multi([parts[1], parts[0]], dtype, devop, arg, n_pre_op_srcs=2,
                                      post_op=last and devop == 4)[0]
        else:
            acc = oracle.reduce_multi([parts[k], acc], dtype, devop, arg, n_pre_op_srcs=1,
                                      post_op=last and devop == 4)[0]
    return acc


@pytest.mark.parametrize("n,grid", [(2, ""), (3, ""), (3, "2"), (8, ""), (8, "3")])
def test_multiprocess_ring_fifo_reduce_scatter_and_reduce(nbx, oracle, n, grid, monkeypatch):
    """NCCL_ALGO=Ring: ReduceScatter block b folded along the ring b+1, ..., b
    and Reduce along the chain root+1, ..., root, through the step FIFO —
    bitwise NCCL's operand order (ring_chain). NBX_SIMPLE_MAX_GRID=2/3 with
    4 KiB staging slices makes every call run many rounds, so the 2 staging
    slots wrap and the credits gate the producer."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NCCL_ALGO", "Ring")
    monkeypatch.setenv("NCCL_PROTO", "Simple")
    monkeypatch.setenv("NBX_SIMPLE_MAX_GRID", grid or "32")
    monkeypatch.setenv("NBX_SIMPLE_SLICE_BYTES", "4096" if grid else "")
    res = _run_ranks(nbx, n, _child_ring_fifo)
    for i, (kind, dtype, op, count, root) in enumerate(RING_FIFO_CASES):
        root = root % n
        xs = [_ring_fifo_input(kind, dtype, count, n, r) for r in range(n)]
        devop, arg = oracle.host_to_dev_redop(op, dtype, n)
        exp = {}
        if kind == "rs":
            for b in range(n):
                order = [(b + 1 + k) % n for k in range(n)]
                exp[b] = ring_chain(oracle, [xs[j][b * count:(b + 1) * count] for j in order], dtype, devop, arg, n)
        else:
            order = [(root + 1 + k) % n for k in range(n)]
            exp[root] = ring_chain(oracle, [xs[j] for j in order], dtype, devop, arg, n)
        for it in range(2):
            for r, e in exp.items():
                got = res[r][(it, i)]
                if not np.array_equal(got, np.ascontiguousarray(e).view(np.uint8)):
                    w = np.nonzero(got.reshape(-1, e.itemsize) != np.ascontiguousarray(e).view(np.uint8).reshape(
                        -1, e.itemsize))[0] if got.size == e.nbytes else np.array([-1])
                    raise AssertionError(f"ring FIFO iteration {it} {(kind, dtype, op, count, root)} rank {r}: "
                                         f"{np.unique(w).size} of {e.size} elements wrong, first {int(w[0])} last "
                                         f"{int(w[-1])} (fold order ring_chain; NCCL_ALGO=Ring, grid {grid or 32})")


# config D at full size (8 ranks x 1 GiB, direct and ring) and config E:
# tests/test_configs_gpu.py


# (kind, dtype, op, count, byte offset of send/recv). By default slots
# <= 64 KiB take the LL protocol; LL128 up to 1 MiB: one-shot (AllReduce with
# > 2 ranks: up to 256 KiB), LL128 two-shot AllReduce above that; the rest the
# direct (Simple) path. With NCCL_PROTO=LL128 (and a 4 MiB LL128 max) every
# message up to 4 MiB takes LL128. Reduce to a changing root back to back exercises
# the done-word credits (a non-root never waits for data, so only the credits
# stop it from overwriting a slot the root has not read yet).
LL_CASES = [
    ("ar", 7, 0, 1, 0), ("ar", 7, 0, 3, 0), ("ar", 7, 0, 1000, 0), ("ar", 7, 0, 16384, 0), ("ar", 6, 0, 17, 0),
    ("ar", 9, 4, 4097, 0), ("ar", 2, 4, 999, 0), ("ar", 4, 2, 4096, 0), ("ar", 10, 0, 33, 0),
    ("ar", 1, 3, 65536, 0), ("ar", 8, 1, 8191, 0), ("ar", 7, 0, 40000, 0), ("ar", 7, 0, 1001, 4),
    ("ar", 0, 0, 77, 3), ("rs", 7, 0, 1000, 0), ("rs", 6, 4, 333, 2), ("rs", 0, 2, 5, 1), ("rs", 4, 4, 4096, 0),
    ("rs", 7, 0, 20000, 0), ("red", 7, 0, 1000, 0), ("red", 9, 4, 777, 0), ("red", 2, 3, 64, 0),
    ("red", 7, 0, 123, 4), ("red", 7, 1, 4096, 0), ("ar", 7, 0, 64, 0),
    # LL128 one-shot range: odd lengths so 48-byte lines straddle 16-byte blocks
    ("ar", 7, 0, 50003, 0), ("ar", 6, 4, 77777, 2), ("ar", 4, 2, 30000, 8), ("rs", 7, 0, 30001, 4),
    ("rs", 2, 2, 131072, 0), ("red", 7, 0, 99999, 0), ("red", 8, 4, 100000, 8),
    # LL128 two-shot AllReduce / Reduce (> 256 KiB with > 2 ranks; one-shot with 2 ranks)
    ("ar", 7, 4, 262144, 0), ("ar", 9, 0, 300001, 0), ("ar", 11, 0, 600001, 1), ("ar", 7, 0, 300000, 4),
    ("ar", 2, 2, 1000003, 0), ("ar", 8, 0, 200001, 0), ("red", 7, 0, 300001, 0), ("red", 9, 4, 200003, 2),
    ("red", 2, 3, 500000, 0),
    # direct (Simple) path interleaved: > 4 MiB per slot (> 1 MiB by default)
    ("ar", 7, 0, 1100000, 0), ("rs", 7, 4, 1048577, 0),
]


def _ll_input(kind, dtype, count, n, r):
    from oracle import oracle
    total = count * n if kind == "rs" else count
    # source s is seeded by seed + s alone: ranks 0-7 get the same input at any n
    return oracle.random_inputs(dtype, max(8, n), total, seed=77 + dtype + count)[r]


def _ll_root(i, n):
    return (i * 3 + 1) % n


def _child_ll(uid_bytes, rank, n, q, proto):
    try:
        import os
        if proto:
            os.environ["NCCL_PROTO"] = proto
            os.environ["NBX_LL128_MAX_BYTES"] = str(4 << 20)   # the 1-4 MiB cases through both LL128 shapes too
        import time

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        lib = nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        settings = mp_diag.comm_settings(nbx, comm)
        st = torch.cuda.current_stream().cuda_stream
        out = {}
        for it in range(3):   # repeated: exercises both LL parities and LL/direct interleaving
            keep = []
            for i, (kind, dtype, op, count, shift) in enumerate(LL_CASES):
                x = _ll_input(kind, dtype, count, n, rank).view(np.uint8)
                tx = torch.zeros(x.size + 16, dtype=torch.uint8, device="cuda")
                tx[shift:shift + x.size] = torch.from_numpy(x.copy()).cuda()
                out_bytes = x.size // n if kind == "rs" else x.size
                ty = torch.zeros(out_bytes + 16, dtype=torch.uint8, device="cuda")
                sp, rp = tx.data_ptr() + shift, ty.data_ptr() + shift
                if kind == "ar":
                    comm.all_reduce(sp, rp, count, dtype, op, st)
                elif kind == "rs":
                    comm.reduce_scatter(sp, rp, count, dtype, op, st)
                else:
                    comm.reduce(sp, rp, count, dtype, op, _ll_root(i, n), st)
                keep.append((i, ty, shift, out_bytes))   # no sync between calls: ranks run ahead
            torch.cuda.synchronize()
            for i, ty, shift, nb in keep:
                out[(it, i)] = ty[shift:shift + nb].cpu().numpy().copy()
        # latency of a 4 KiB fp32 AllReduce (LL): 200 back-to-back calls
        tx = torch.rand(1024, device="cuda")
        ty = torch.empty_like(tx)
        for _ in range(20):
            comm.all_reduce(tx.data_ptr(), ty.data_ptr(), 1024, 7, 0, st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            comm.all_reduce(tx.data_ptr(), ty.data_ptr(), 1024, 7, 0, st)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) * 1e6 / 200
        err = comm.async_error()   # a device check that failed (NBX_CHECK_SLICES / plans) names itself here
        assert err == 0, (err, (lib.ncclGetLastError(None) or b"").decode(errors="replace"))
        comm.destroy()
        q.put((rank, "ok", (out, us, settings)))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("n,proto,checks", [(2, "", ""), (3, "", ""), (5, "", ""), (2, "LL128", ""), (3, "LL128", ""),
                                            (8, "", ""), (8, "", "slices"), (8, "", "ring")])
def test_multiprocess_ll_protocol(nbx, oracle, n, proto, checks, monkeypatch):
    """LL protocol (one kernel, {data, flag} 8-byte lines, no host exchange) for
    small, LL128 (120 payload bytes + flag per 128-byte line) for medium
    AllReduce / ReduceScatter / Reduce messages, misaligned buffers included,
    issued back to back without host synchronisation and interleaved with each
    other and with direct-path messages; bitwise equal to the direct schedule's
    fold order. NCCL_PROTO=LL128 routes every message that fits through LL128.
    checks="slices": the 8-rank run of GPUTEST_r05's red record with every
    Simple hand-off verified by its slice checksum (NBX_CHECK_SLICES=1);
    checks="ring": the same with the Simple-sized calls on the ring schedule
    (NCCL_ALGO=Ring: for these commutative ops NCCL's ring chain gives the
    direct schedule's bits)."""
    monkeypatch.setenv("NBX_CHECK_SLICES", "1" if checks == "slices" else "")
    monkeypatch.setenv("NCCL_ALGO", "Ring" if checks == "ring" else "")
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    # all ranks share the test box's one GPU: keep every rank's LL128 grid
    # co-resident (8 ranks x 16 workgroups), as one GPU per rank guarantees
    monkeypatch.setenv("NBX_LL128_MAX_GRID", "16")
    uid = nbx.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_child_ll, args=(bytes(uid), r, n, q, proto), daemon=True) for r in range(n)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(n):
            rank, status, payload = q.get(timeout=300)
            assert status == "ok", f"rank {rank}:\n{payload}"
            res[rank] = payload
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
    failures = []   # every wrong output of every case, rank and iteration, described at the end
    for i, (kind, dtype, op, count, shift) in enumerate(LL_CASES):
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
        for it in range(3):
            for r, e in exp.items():
                got = res[r][0][(it, i)]
                if not np.array_equal(got, np.ascontiguousarray(e).view(np.uint8)):
                    failures.append((f"case {i} {LL_CASES[i]} iteration {it}", kind, dtype, op, count, r, got, xs,
                                     res[r][2], _ll_root(i, n)))
    mp_diag.raise_collective_failures(oracle, failures, n, what=f"NCCL_PROTO={proto or 'default'}: ")
    print(f"LL 4 KiB fp32 allreduce (NCCL_PROTO={proto or 'default'}), {n} ranks sharing one GPU: us/call =",
          [round(res[r][1], 1) for r in range(n)])


# fp32 counts -> protocol by default (2-3 ranks): LL, LL128 one-shot, LL128
# two-shot (3 ranks; one-shot at 2), Simple
GRAPH_CASES = [(1000, "LL"), (50003, "LL128"), (200001, "LL128 two-shot"), (1500000, "Simple"),
               # one ncclGroupStart/End: two LL-sized calls and two LL128 one-shot calls -> two group launches
               (777, "LL group"), (4099, "LL group"), (20000, "LL128 group"), (30001, "LL128 group")]


def _child_graph(uid_bytes, uid_ring_bytes, rank, n, q):
    """Capture one graph holding AllReduce calls of every protocol (direct
    comm) plus a ring-schedule AllReduce (ring comm), replay it with inputs
    changed between replays, check every output each time."""
    try:
        import os

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        os.environ["NCCL_ALGO"] = "Ring"
        os.environ["NCCL_PROTO"] = "Simple"
        ring = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_ring_bytes), rank)
        s = torch.cuda.Stream()
        bufs = []
        for cnt, _ in GRAPH_CASES + [(300001, "ring")]:
            x = torch.empty(cnt, device="cuda")
            y = torch.empty(cnt, device="cuda")
            bufs.append((cnt, x, y))

        labels = [lab for _, lab in GRAPH_CASES] + ["ring"]

        def issue(st):
            grouped = False
            for i, (cnt, x, y) in enumerate(bufs):
                if labels[i].endswith("group") and not grouped:
                    nbx.group_start()
                    grouped = True
                elif not labels[i].endswith("group") and grouped:
                    nbx.group_end()
                    grouped = False
                c = ring if i == len(bufs) - 1 else comm
                c.all_reduce(x.data_ptr(), y.data_ptr(), cnt, 7, 0, st)
            if grouped:
                nbx.group_end()

        def fill(it):
            for cnt, x, y in bufs:
                idx = torch.arange(cnt, device="cuda", dtype=torch.float32)
                x.copy_(torch.remainder(idx * 3 + 11 * rank + 17 * it, 257))
                y.fill_(-1)

        with torch.cuda.stream(s):
            fill(0)
            issue(s.cuda_stream)   # eager warm-up: maps every peer buffer before capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
            issue(s.cuda_stream)
        torch.cuda.synchronize()
        bad = []
        for it in range(1, 6):
            with torch.cuda.stream(s):
                fill(it)
                g.replay()
            s.synchronize()
            for k, (cnt, x, y) in enumerate(bufs):
                idx = torch.arange(cnt, device="cuda", dtype=torch.float32)
                want = sum(torch.remainder(idx * 3 + 11 * r + 17 * it, 257) for r in range(n))
                if not torch.equal(y, want):
                    bad.append((it, k, int((y != want).sum())))
        # eager calls after the replays still line up with the peers
        with torch.cuda.stream(s):
            fill(9)
            issue(s.cuda_stream)
        s.synchronize()
        for k, (cnt, x, y) in enumerate(bufs):
            idx = torch.arange(cnt, device="cuda", dtype=torch.float32)
            want = sum(torch.remainder(idx * 3 + 11 * r + 17 * 9, 257) for r in range(n))
            if not torch.equal(y, want):
                bad.append(("eager", k, int((y != want).sum())))
        assert comm.async_error() == 0 and ring.async_error() == 0
        del g
        ring.destroy()
        comm.destroy()
        q.put((rank, "ok", bad))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("n", [2, 3])
def test_multiprocess_graph_capture(nbx, n, monkeypatch):
    """ncclAllReduce captured into a HIP graph on the multi-process communicator
    (LL, LL128, Simple direct and ring schedules in one graph) replays
    correctly: sequence numbers, credits and barrier epochs are device-resident,
    so every replay advances them like an eager call."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NBX_LL128_MAX_GRID", "16")
    monkeypatch.delenv("NCCL_PROTO", raising=False)
    monkeypatch.delenv("NCCL_ALGO", raising=False)
    uid, uid_ring = nbx.get_unique_id(), nbx.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_child_graph, args=(bytes(uid), bytes(uid_ring), r, n, q), daemon=True)
             for r in range(n)]
    for p in procs:
        p.start()
    try:
        for _ in range(n):
            rank, status, payload = q.get(timeout=300)
            assert status == "ok", f"rank {rank}:\n{payload}"
            assert payload == [], f"rank {rank}: wrong outputs {payload}"
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()


def _child_failure(uid_bytes, rank, q, evq):
    """Rank 0 meets an absent peer: the LL kernel's and the Simple kernel's
    bounded spins time out (ncclRemoteError via ncclCommGetAsyncError), and
    ncclCommAbort ends a spinning kernel at once. Rank 1 joins the communicator and then
    issues nothing until rank 0 is done."""
    try:
        import time

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(2, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        if rank == 1:
            evq.get(timeout=240)   # rank 0 finished
            comm.destroy()
            q.put((rank, "ok", None))
            return
        st = torch.cuda.current_stream().cuda_stream
        out = {}
        x = torch.ones(1024, device="cuda")
        y = torch.empty_like(x)
        t0 = time.perf_counter()
        comm.all_reduce(x.data_ptr(), y.data_ptr(), 1024, 7, 0, st)   # LL: the kernel spins, then times out
        torch.cuda.synchronize()
        out["ll_timeout_s"] = time.perf_counter() - t0
        out["ll_async_error"] = comm.async_error()
        big = torch.ones(4 << 20, device="cuda")   # 16 MiB: Simple protocol kernel
        t0 = time.perf_counter()
        comm.all_reduce(big.data_ptr(), big.data_ptr(), big.numel(), 7, 0, st)
        torch.cuda.synchronize()
        out["simple_timeout_s"] = time.perf_counter() - t0
        out["simple_error"] = comm.async_error()
        comm.abort()
        # a fresh communicator whose peer never calls: abort ends the spinning kernel
        evq.put("next")
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def _child_selftest(uid_bytes, rank, n, q):
    try:
        import ctypes

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        lib = nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        lib.nbxDebugCommProtoMask.argtypes = [ctypes.c_void_p]
        lib.nbxDebugCommProtoMask.restype = ctypes.c_int
        mask = lib.nbxDebugCommProtoMask(comm.handle)
        st = torch.cuda.current_stream().cuda_stream
        bad = 0
        for cnt in (30000, 300001):   # LL128 one-shot / two-shot sizes (Simple without LL128)
            idx = torch.arange(cnt, device="cuda", dtype=torch.float32)
            x = torch.remainder(idx * 3 + 11 * rank, 257)
            y = torch.empty_like(x)
            comm.all_reduce(x.data_ptr(), y.data_ptr(), cnt, 7, 0, st)
            torch.cuda.synchronize()
            want = sum(torch.remainder(idx * 3 + 11 * r, 257) for r in range(n))
            bad += int((y != want).sum())
        comm.destroy()
        q.put((rank, "ok", (mask, bad)))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("tear,delay_us", [(0, 0), (1, 200), (1, 5000)])
def test_ll128_torn_line_is_waited_on(nbx, torch_gpu, tear, delay_us):
    """A deliberately torn LL128 line (nbxDebugLL128TearTest: the writer stores
    the line's last 32 bytes — the flag half of the r1 one-flag layout — waits,
    then the first 32 bytes) against the collectives' own line reader: with a
    flag in every 16-byte chunk the reader waits for the second half and folds
    exactly the new payload, never the stale chunks."""
    import ctypes
    lib = nbx.load_library()
    lib.nbxDebugLL128TearTest.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_longlong)]
    lib.nbxDebugLL128TearTest.restype = ctypes.c_int
    after = ctypes.c_longlong(0)
    rc = lib.nbxDebugLL128TearTest(delay_us, tear, ctypes.byref(after))
    assert rc == 0, {1: "stale chunks folded", 2: "accepted before the second half", 3: "reader timed out"}.get(rc, rc)
    if tear:
        assert after.value >= 0   # accepted after the second half was issued (100 MHz ticks)


@pytest.mark.parametrize("n,fail", [(3, False), (3, True), (8, False)])
def test_multiprocess_ll128_selftest(nbx, monkeypatch, n, fail):
    """ncclCommInitRank probes LL128 (AllReduces checked exactly) before using
    it; a failed probe on any rank drops LL128 on every rank (simulated with
    NBX_LL128_SELFTEST_FAIL=1) and the LL128-sized calls still come out right
    on the Simple path. 8 ranks: the rank count whose probe failed init in r1
    (profiles/r1/pytest_gpu_r1s.log), forced on the shared GPU."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NBX_LL128_MAX_GRID", "16")
    monkeypatch.delenv("NCCL_PROTO", raising=False)
    monkeypatch.delenv("NCCL_ALGO", raising=False)
    monkeypatch.setenv("NBX_LL128_SELFTEST_ITERS", "8")   # forced: the ranks share one GPU here
    if fail:
        monkeypatch.setenv("NBX_LL128_SELFTEST_FAIL", "1")
    else:
        monkeypatch.delenv("NBX_LL128_SELFTEST_FAIL", raising=False)
    res = _run_ranks(nbx, n, _child_selftest)
    for r in range(n):
        mask, bad = res[r]
        assert bad == 0, (r, bad)
        assert mask == (5 if fail else 7), (r, mask)   # LL|Simple after a failed probe, else all three


@pytest.mark.parametrize("proto,override,want", [("", "", 5), ("LL128,LL,Simple", "", 7), ("", "1", 7)])
def test_multiprocess_ll128_gate_across_gpus(nbx, monkeypatch, proto, override, want):
    """Ranks that report different GPUs (NBX_DEBUG_ASSUME_MULTI_GPU=1: the gate
    only, not the grid split) start without LL128, as the reference enables
    LL128 by default only on validated fabrics (tuning.cc:287-297): the
    LL128-sized calls run on Simple, exact. NCCL_PROTO naming LL128, or
    NBX_LL128_ACROSS_GPUS=1, keeps it (and its creation-time probe runs)."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NBX_LL128_MAX_GRID", "16")
    monkeypatch.setenv("NBX_DEBUG_ASSUME_MULTI_GPU", "1")
    monkeypatch.setenv("NCCL_PROTO", proto)
    monkeypatch.setenv("NBX_LL128_ACROSS_GPUS", override)
    monkeypatch.setenv("NBX_LL128_SELFTEST_ITERS", "4")
    monkeypatch.delenv("NCCL_ALGO", raising=False)
    monkeypatch.delenv("NBX_LL128_SELFTEST_FAIL", raising=False)
    res = _run_ranks(nbx, 3, _child_selftest)
    for r in range(3):
        mask, bad = res[r]
        assert bad == 0, (r, bad)
        assert mask == want, (r, mask)


def _child_abort(uid_bytes, rank, q, evq):
    try:
        import threading
        import time

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(2, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        if rank == 1:
            evq.get(timeout=240)
            comm.destroy()
            q.put((rank, "ok", None))
            return
        st = torch.cuda.current_stream().cuda_stream
        x = torch.ones(1024, device="cuda")
        comm.all_reduce(x.data_ptr(), x.data_ptr(), 1024, 7, 0, st)   # spins: the peer never arrives
        time.sleep(0.5)
        t0 = time.perf_counter()
        comm.abort()   # sets the abort word, waits for the device, frees
        torch.cuda.synchronize()
        evq.put("done")
        q.put((rank, "ok", {"abort_s": time.perf_counter() - t0}))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_multiprocess_timeout_and_abort(nbx, monkeypatch):
    """Failure handling with a peer that never arrives: bounded spins end with
    ncclRemoteError (kernel path: async error; host exchange: the call's return
    code) after NBX_TIMEOUT_SEC, and ncclCommAbort ends a spinning kernel in
    well under that timeout."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "3")
    ctx = mp.get_context("spawn")
    for child, check in ((_child_failure, "failure"), (_child_abort, "abort")):
        if check == "abort":
            monkeypatch.setenv("NBX_TIMEOUT_SEC", "120")
        uid = nbx.get_unique_id()
        q, evq = ctx.Queue(), ctx.Queue()
        procs = [ctx.Process(target=child, args=(bytes(uid), r, q, evq), daemon=True) for r in range(2)]
        for p in procs:
            p.start()
        res = {}
        try:
            for _ in range(2):
                rank, status, payload = q.get(timeout=300)
                assert status == "ok", f"{check} rank {rank}:\n{payload}"
                res[rank] = payload
            for p in procs:
                p.join(timeout=60)
        finally:
            for p in procs:
                if p.is_alive():
                    p.terminate()
        r0 = res[0]
        if check == "failure":
            assert r0["ll_async_error"] == 6, r0          # ncclRemoteError
            assert 2.5 < r0["ll_timeout_s"] < 30, r0
            assert r0["simple_error"] == 6, r0
            assert 2.5 < r0["simple_timeout_s"] < 30, r0
        else:
            assert r0["abort_s"] < 20, r0                 # not the 120 s timeout


# Float min/max with ±0 ties and NaNs: a tie returns the
# second operand (oracle/reduce_oracle.c header), so the operand order of every
# fold step is observable. Direct schedules fold Fn(acc, next) in the order
# b+1, ..., b; ring / chain hops fold Fn(local, received) (ring_chain above).
TIE_BITS = {   # +0, -0, +1, -1, +inf, -inf, qNaN, 2.5 (zeros drawn most often)
    7: (np.uint32, [0x0, 0x80000000, 0x3f800000, 0xbf800000, 0x7f800000, 0xff800000, 0x7fc00000, 0x40200000]),
    8: (np.uint64, [0x0, 1 << 63, 0x3ff0000000000000, 0xbff0000000000000, 0x7ff0000000000000,
                    0xfff0000000000000, 0x7ff8000000000000, 0x4004000000000000]),
    6: (np.uint16, [0x0, 0x8000, 0x3c00, 0xbc00, 0x7c00, 0xfc00, 0x7e00, 0x4100]),
    9: (np.uint16, [0x0, 0x8000, 0x3f80, 0xbf80, 0x7f80, 0xff80, 0x7fc0, 0x4020]),
}
TIE_CASES = [(kind, dt, op) for kind in ("ar", "rs", "red") for dt in (7, 8, 6, 9) for op in (2, 3)]
TIE_COUNT = 6007


def _tie_input(kind, dt, op, n, r):
    st, bits = TIE_BITS[dt]
    total = TIE_COUNT * n if kind == "rs" else TIE_COUNT
    rng = np.random.default_rng(9000 + 100 * dt + 10 * op + r + (0 if kind == "ar" else 3 if kind == "rs" else 6))
    pick = rng.choice(len(bits), size=total, p=[0.3, 0.3, 0.06, 0.06, 0.06, 0.06, 0.1, 0.06])
    return np.array(bits, dtype=st)[pick]


def _child_ties(uid_direct, rank, n, q, uid_ring):
    try:
        import os

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        os.environ["NCCL_PROTO"] = "Simple"
        comms = {"direct": nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_direct), rank)}
        os.environ["NCCL_ALGO"] = "Ring"
        comms["ring"] = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_ring), rank)
        st = torch.cuda.current_stream().cuda_stream
        out = {}
        for algo, comm in comms.items():
            for i, (kind, dt, op) in enumerate(TIE_CASES):
                x = _tie_input(kind, dt, op, n, rank)
                tx = torch.from_numpy(x.view(np.uint8).copy()).cuda()
                nb = TIE_COUNT * x.itemsize
                ty = torch.zeros(nb, dtype=torch.uint8, device="cuda")
                root = i % n
                if kind == "ar":
                    comm.all_reduce(tx.data_ptr(), ty.data_ptr(), TIE_COUNT, dt, op, st)
                elif kind == "rs":
                    comm.reduce_scatter(tx.data_ptr(), ty.data_ptr(), TIE_COUNT, dt, op, st)
                else:
                    comm.reduce(tx.data_ptr(), ty.data_ptr() if rank == root else 0, TIE_COUNT, dt, op, root, st)
                torch.cuda.synchronize()
                out[(algo, i)] = ty.cpu().numpy().copy()
            assert comm.async_error() == 0
        for comm in comms.values():
            comm.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("n", [2, 3])
def test_multiprocess_float_minmax_ties(nbx, oracle, n, monkeypatch):
    """f32 / f64 / f16 / bf16 ncclMax and ncclMin over inputs that are mostly
    ±0 with NaNs and infinities, AllReduce / ReduceScatter / Reduce, on the
    direct and the ring schedule: bit-exact against the oracle folded in each
    schedule's own operand order (direct: left fold b+1, ..., b; ring: NCCL's
    hop order Fn(local, received) along the chain b+1 -> ... -> b)."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NBX_SIMPLE_MAX_GRID", "8")
    res = _run_ranks(nbx, n, _child_ties, bytes(nbx.get_unique_id()))
    for i, (kind, dt, op) in enumerate(TIE_CASES):
        xs = [_tie_input(kind, dt, op, n, r) for r in range(n)]
        xs = [x.view(oracle.NP_STORAGE[dt]) for x in xs]
        devop, arg = oracle.host_to_dev_redop(op, dt, n)
        eb = xs[0].itemsize
        root = i % n
        for algo in ("direct", "ring"):
            def fold(parts):
                if algo == "direct":
                    return oracle.reduce_multi(parts, dt, devop, arg, n_pre_op_srcs=n)[0]
                return ring_chain(oracle, parts, dt, devop, arg, n)
            exp = {}
            if kind == "rs":
                for b in range(n):
                    exp[b] = fold([xs[(b + 1 + k) % n][b * TIE_COUNT:(b + 1) * TIE_COUNT] for k in range(n)])
            elif kind == "ar":
                full = np.empty(TIE_COUNT, dtype=xs[0].dtype)
                for c, (lo, hi) in enumerate(_blocks(TIE_COUNT, eb, n)):
                    if hi > lo:
                        full[lo:hi] = fold([xs[(c + 1 + k) % n][lo:hi] for k in range(n)])
                exp = {r: full for r in range(n)}
            else:
                exp[root] = fold([xs[(root + 1 + k) % n] for k in range(n)])
            for r, e in exp.items():
                got = res[r][(algo, i)]
                mp_diag.check_equal(got, np.ascontiguousarray(e).view(np.uint8), (algo, kind, dt, op, r))


def _child_streams(uid_bytes, rank, n, q):
    """Successive calls of one communicator alternate between two streams with
    no ordering by the caller: the library orders them (the Simple /
    ring kernels share the communicator's device-resident counters)."""
    try:
        import os

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        os.environ["NCCL_PROTO"] = "Simple"
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        outs = []
        for it in range(8):
            s = streams[it % 2]
            cnt = 300001 + 4096 * it
            with torch.cuda.stream(s):
                idx = torch.arange(cnt, device="cuda", dtype=torch.float32)
                x = torch.remainder(idx * 3 + 11 * rank + it, 257)
                y = torch.full((cnt,), -1.0, device="cuda")
                comm.all_reduce(x.data_ptr(), y.data_ptr(), cnt, 7, 0, s.cuda_stream)
            outs.append((it, cnt, x, y))
        # a call on a raw stream destroyed right after it (its work still
        # queued), then calls on another stream: the next call waits on the
        # event recorded behind the destroyed stream's call (hipStreamDestroy
        # waited for that work), never touching the dead stream itself
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so.7")
        hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
        torch.cuda.synchronize()
        for it in range(8, 11):
            cnt = 300001 + 4096 * it
            idx = torch.arange(cnt, device="cuda", dtype=torch.float32)
            x = torch.remainder(idx * 3 + 11 * rank + it, 257)
            y = torch.full((cnt,), -1.0, device="cuda")
            torch.cuda.synchronize()
            if it == 9:
                raw = ctypes.c_void_p()
                assert hip.hipStreamCreateWithFlags(ctypes.byref(raw), 1) == 0
                comm.all_reduce(x.data_ptr(), y.data_ptr(), cnt, 7, 0, raw.value)
                assert hip.hipStreamDestroy(raw) == 0
            else:
                comm.all_reduce(x.data_ptr(), y.data_ptr(), cnt, 7, 0, streams[0].cuda_stream)
            outs.append((it, cnt, x, y))
        torch.cuda.synchronize()
        bad = []
        for it, cnt, x, y in outs:
            idx = torch.arange(cnt, device="cuda", dtype=torch.float32)
            want = sum(torch.remainder(idx * 3 + 11 * r + it, 257) for r in range(n))
            if not torch.equal(y, want):
                bad.append((it, int((y != want).sum())))
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", bad))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("n", [2, 3])
def test_multiprocess_calls_alternate_streams(nbx, n, monkeypatch):
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NBX_SIMPLE_MAX_GRID", "8")
    res = _run_ranks(nbx, n, _child_streams)
    for r in range(n):
        assert res[r] == [], (r, res[r])


def _child_nonblocking(uid_bytes, rank, n, q):
    """Non-blocking communicator (config.blocking = 0): ncclCommInitRankConfig
    returns ncclInProgress at once, operations before the initialisation has
    finished fail with ncclInvalidArgument (ncclCommEnsureReady,
    init.cc:287-305), ncclCommGetAsyncError turns ncclSuccess, then the
    communicator works like a blocking one."""
    try:
        import time

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        if rank != 0:
            time.sleep(1.5)   # rank 0's initialisation cannot finish before this
        uid = nbx.ncclUniqueId.from_buffer_copy(uid_bytes)
        comm, rc = nbx.Communicator.init_rank_config(n, uid, rank, blocking=0)
        early = []
        assert rc == int(nbx.ncclResult.ncclInProgress), rc
        if rank == 0:
            for name, fn in (("count", lambda: comm.count()),
                             ("all_reduce", lambda: comm.all_reduce(0, 0, 16, 7, 0, 0))):
                try:
                    fn()
                    early.append((name, "succeeded"))
                except nbx.NcclError as e:
                    early.append((name, int(e.code)))
        t0 = time.monotonic()
        while comm.async_error() == int(nbx.ncclResult.ncclInProgress):
            assert time.monotonic() - t0 < 120, "initialisation did not finish"
            time.sleep(0.01)
        final = comm.async_error()
        cnt = 100003
        x = torch.remainder(torch.arange(cnt, device="cuda", dtype=torch.float32) * 5 + rank, 97)
        y = torch.full((cnt,), -1.0, device="cuda")
        comm.all_reduce(x.data_ptr(), y.data_ptr(), cnt, 7, 0, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        want = sum(torch.remainder(torch.arange(cnt, device="cuda", dtype=torch.float32) * 5 + r, 97) for r in range(n))
        ok = bool(torch.equal(y, want))
        comm.destroy()
        q.put((rank, "ok", {"early": early, "final": final, "exact": ok, "count_after": n}))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("n", [2, 3])
def test_multiprocess_nonblocking_init(nbx, n, monkeypatch):
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    res = _run_ranks(nbx, n, _child_nonblocking)
    inval = int(nbx.ncclResult.ncclInvalidArgument)
    assert res[0]["early"] == [("count", inval), ("all_reduce", inval)], res[0]
    for r in range(n):
        assert res[r]["final"] == 0 and res[r]["exact"], (r, res[r])


# Groups of LL-sized (and LL128 one-shot sized) calls run as ONE launch per run
# of compatible calls (comm_mp_launch.cc runMpGroup / runMpLLGroup): (kind, dtype,
# op, count, stream).
# Runs are cut by kind / type / op / root changes, by the LL slot capacity
# (64 KiB: the 16 x 4096-float AllReduces need four launches) and by the
# 16-segment limit (the 40 x 10-element AllReduces: 16 + 16 + 8); stream 1
# inside a run exercises the fan-in / fan-out across the rank's streams.
GROUP_SMALL = ([("allreduce", 7, 0, c, 0) for c in (1, 7, 1000, 4099, 3)] + [("allreduce", 7, 0, 513, 1)] +
               [("allreduce", 6, 4, c, 0) for c in (33, 2048, 9)] +
               [("reducescatter", 2, 0, c, 0) for c in (5, 100, 1000, 17)] +
               [("reduce", 9, 2, c, 0) for c in (77, 4000, 1)] +
               [("allreduce", 7, 0, 4096, i % 2) for i in range(16)] +
               [("allreduce", 8, 1, 10, 0) for _ in range(40)] +
               # LL128 one-shot runs (64 KiB < slot <= 256 KiB per call)
               [("allreduce", 7, 0, c, i % 2) for i, c in enumerate((30000, 17001, 60000, 20000, 40000, 33333))] +
               [("reducescatter", 2, 3, c, 0) for c in (20000, 17003, 30000)] +
               [("reduce", 4, 0, c, 0) for c in (20000, 9001)])


def _small_inputs(oracle, k, kind, dtype, count, n, r):
    cnt = count * n if kind == "reducescatter" else count
    return oracle.random_inputs(dtype, n, cnt, seed=5000 + 7 * k)[r]


# Simple-sized groups (run with NCCL_PROTO=Simple): runs of one kind / type /
# op become ONE Simple launch (SimpleSeg), cut at 16 calls, at kind / type /
# op / root changes and where a call reads what an earlier one of the run
# writes; sizes with partial slices, ragged blocks and one-element messages.
GROUP_SIMPLE = ([("allreduce", 7, 0, c, 0) for c in (300000, 1, 40009, 1 << 20, 17, 70000)] +
                [("allreduce", 7, 0, 5000 + i, i % 2) for i in range(20)] +
                [("allreduce", 9, 0, c, 0) for c in (40000, 1023, 200001)] +
                [("reducescatter", 2, 2, c, 0) for c in (100000, 3, 65536)] +
                [("reduce", 4, 3, c, 0) for c in (77777, 1, 300000)] +
                [("allreduce", 6, 4, c, 0) for c in (33333, 99999)])


def _child_group_small(uid_bytes, rank, n, q, which="small"):
    cases = GROUP_SIMPLE if which == "simple" else GROUP_SMALL
    try:
        import torch
        from tests.conftest import load_package
        from oracle import oracle
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        out = {}
        for it in range(2):
            live = []
            nbx.group_start()
            for k, (kind, dtype, op, count, si) in enumerate(cases):
                x = _small_inputs(oracle, k, kind, dtype, count, n, rank)
                tx = torch.from_numpy(x.view(np.uint8).copy()).cuda()
                ty = torch.full((count * x.itemsize,), 0xAB, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                s = streams[si].cuda_stream
                if kind == "allreduce":
                    comm.all_reduce(tx.data_ptr(), ty.data_ptr(), count, dtype, op, s)
                elif kind == "reducescatter":
                    comm.reduce_scatter(tx.data_ptr(), ty.data_ptr(), count, dtype, op, s)
                else:
                    comm.reduce(tx.data_ptr(), ty.data_ptr() if rank == 1 % n else 0, count, dtype, op, 1 % n, s)
                live.append((k, tx, ty))
            nbx.group_end()
            torch.cuda.synchronize()
            for k, tx, ty in live:
                out[(it, k)] = ty.cpu().numpy().copy()
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("n,batch,which,algo", [(2, "1", "small", ""), (3, "1", "small", ""), (3, "0", "small", ""),
                                                 (2, "1", "simple", ""), (3, "1", "simple", ""),
                                                 (4, "1", "simple", "Ring"), (3, "0", "simple", "")])
def test_multiprocess_grouped_small_calls_one_launch(nbx, oracle, n, batch, which, algo, monkeypatch):
    """Bit-exact vs the oracle in the direct schedule's order, batched into
    group launches (NBX_GROUP_BATCH=1, default) and one kernel per call (0):
    LL / LL128 runs ("small"), and Simple runs ("simple", NCCL_PROTO=Simple;
    direct and ring schedules — for the commutative ops tested the ring's
    order gives the same bits)."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NBX_LL_MAX_GRID", "64")
    monkeypatch.setenv("NBX_GROUP_BATCH", batch)
    monkeypatch.setenv("NCCL_PROTO", "Simple" if which == "simple" else "")
    monkeypatch.setenv("NCCL_ALGO", algo)
    res = _run_ranks(nbx, n, _child_group_small, which)
    for k, (kind, dtype, op, count, si) in enumerate(GROUP_SIMPLE if which == "simple" else GROUP_SMALL):
        xs = [_small_inputs(oracle, k, kind, dtype, count, n, r) for r in range(n)]
        devop, arg = oracle.host_to_dev_redop(op, dtype, n)
        st = oracle.NP_STORAGE[dtype]
        eb = np.dtype(st).itemsize
        blocks = ([(b * count, (b + 1) * count) for b in range(n)] if kind == "reducescatter"
                  else _blocks(xs[0].size, eb, n))
        full = np.empty(xs[0].size, dtype=st)
        for b, (lo, hi) in enumerate(blocks):
            if hi > lo:
                first = (1 % n if kind == "reduce" else b) + 1
                order = [(first + j) % n for j in range(n)]
                full[lo:hi] = oracle.reduce_multi([xs[j][lo:hi] for j in order], dtype, devop, arg,
                                                  n_pre_op_srcs=n, post_op=devop == 4)[0]
        for it in range(2):
            for r in range(n):
                got = res[r][(it, k)].view(st)
                if kind == "allreduce":
                    exp = full
                elif kind == "reducescatter":
                    exp = full[r * count:(r + 1) * count]
                elif r != 1 % n:
                    continue
                else:
                    exp = full
                mp_diag.check_equal(got.view(np.uint8), exp.view(np.uint8), (it, k, kind, dtype, op, count, r))


REDUCE_CHAIN_COUNTS = (1000, 30000, 300000)   # LL, LL128 one-shot, Simple (defaults, one GPU)


def _child_reduce_chain(uid_bytes, rank, n, q, null_recv):
    """a group whose second Reduce reads what the first one writes
    on the root (x -> y, then y -> z; and one buffer reduced in place twice).
    The root's recv is written, a non-root's is not, so a cut that looked at
    each rank's own writes split the root's run and batched the non-roots'.
    Non-roots pass the same pointers as the root, or NULL recv buffers
    (`null_recv`; then the chain reads y, which only the root has)."""
    try:
        import torch
        from tests.conftest import load_package
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        s = torch.cuda.current_stream().cuda_stream
        I32, SUM = 2, 0
        out = {}
        for count in REDUCE_CHAIN_COUNTS:
            i = torch.arange(count, dtype=torch.int32, device="cuda")
            x = (i * 3 + rank * 7) % 101
            y = rank * 1000 + i % 13
            z = torch.full_like(i, -1)
            w = (i * 5 + rank) % 89   # reduced in place twice
            torch.cuda.synchronize()
            recv_y = y.data_ptr() if (rank == 0 or not null_recv) else 0
            recv_z = z.data_ptr() if (rank == 0 or not null_recv) else 0
            nbx.group_start()
            comm.reduce(x.data_ptr(), recv_y, count, I32, SUM, 0, s)
            comm.reduce(y.data_ptr(), recv_z, count, I32, SUM, 0, s)
            comm.reduce(w.data_ptr(), w.data_ptr(), count, I32, SUM, 0, s)
            comm.reduce(w.data_ptr(), w.data_ptr(), count, I32, SUM, 0, s)
            nbx.group_end()
            torch.cuda.synchronize()
            out[count] = (y.cpu().numpy().copy(), z.cpu().numpy().copy(), w.cpu().numpy().copy())
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("n,null_recv", [(2, False), (3, False), (3, True)])
def test_multiprocess_grouped_reduce_chain_root_and_nonroot(nbx, n, null_recv, monkeypatch):
    """Grouped Reduce chains cut alike on the root and the non-roots (a
    Reduce never shares a launch with another call of its group), at LL,
    LL128 and Simple sizes: exact int32 sums, every rank's buffers as NCCL
    leaves them (a non-root's recv untouched)."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "30")
    monkeypatch.setenv("NBX_LL_MAX_GRID", "64")
    res = _run_ranks(nbx, n, _child_reduce_chain, null_recv)
    for count in REDUCE_CHAIN_COUNTS:
        i = np.arange(count, dtype=np.int64)
        xs = [(i * 3 + r * 7) % 101 for r in range(n)]
        ys = [r * 1000 + i % 13 for r in range(n)]
        ws = [(i * 5 + r) % 89 for r in range(n)]
        S = sum(xs)
        Z = S + sum(ys[1:])        # the root's y is S by then; a non-root's y is its own
        W1 = sum(ws)
        W2 = W1 + sum(ws[1:])
        y0, z0, w0 = res[0][count]
        mp_diag.check_equal(y0, S.astype(np.int32), ("y0", count))
        mp_diag.check_equal(z0, Z.astype(np.int32), ("z0", count))
        mp_diag.check_equal(w0, W2.astype(np.int32), ("w0", count))
        for r in range(1, n):
            yr, zr, wr = res[r][count]
            mp_diag.check_equal(yr, ys[r].astype(np.int32), ("y", count, r))
            mp_diag.check_equal(wr, ws[r].astype(np.int32), ("w", count, r))
            assert (zr == -1).all()


def _child_transport(uid_bytes, rank, n, q, count):
    """nbxDebugTransportAllReduce (config D's transport alone): the direct
    schedule's pushes and gather with the fold reduced to a copy of the own
    input, so block j of every rank's output is block j of rank j's input;
    interleaved with real AllReduces on the same communicator (shared
    sequencing and staging), which stay exact."""
    try:
        import ctypes

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        lib = nbx.load_library()
        lib.nbxDebugTransportAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                                   ctypes.c_void_p, ctypes.c_void_p]
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        st = torch.cuda.current_stream().cuda_stream
        idx = torch.arange(count, dtype=torch.int32, device="cuda")
        out = {"xport": [], "ar": []}
        for it in range(3):
            x = ((idx * 7 + rank * 131 + it) % 1000).to(torch.float32)
            y = torch.full_like(x, -1.0)
            rc = lib.nbxDebugTransportAllReduce(x.data_ptr(), y.data_ptr(), count, 7, comm.handle, st)
            z = torch.full_like(x, -1.0)
            comm.all_reduce(x.data_ptr(), z.data_ptr(), count, 7, 0, st)
            torch.cuda.synchronize()
            out["xport"].append((rc, y.cpu().numpy().copy()))
            out["ar"].append(z.cpu().numpy().copy())
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("n,count", [(2, 1 << 20), (3, 300001)])
def test_multiprocess_transport_only_call(nbx, monkeypatch, n, count):
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "30")
    res = _run_ranks(nbx, n, _child_transport, count)
    blocks = _blocks(count, 4, n)
    i = np.arange(count, dtype=np.int64)
    for it in range(3):
        xs = [((i * 7 + r * 131 + it) % 1000).astype(np.float32) for r in range(n)]
        want_x = np.empty(count, np.float32)
        for j, (lo, hi) in enumerate(blocks):
            want_x[lo:hi] = xs[j][lo:hi]
        for r in range(n):
            rc, y = res[r]["xport"][it]
            assert rc == 0
            mp_diag.check_equal(y, want_x, ("xport", r, it))
            mp_diag.check_equal(res[r]["ar"][it], sum(xs), ("ar", r, it))


def _child_link_probe(uid_bytes, rank, n, q):
    """nbxDebugLinkProbe (the fabric rate config D is priced against): push
    and pull launches succeed and report whole passes of at least the asked
    bytes; bad arguments are refused; a Simple-sized AllReduce after it (the
    communicator kept quiet around the probe, as collective_leg.py does) is
    exact although the probe overwrote the staging slices."""
    try:
        import ctypes

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        lib = nbx.load_library()
        lib.nbxDebugLinkProbe.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        st = torch.cuda.current_stream().cuda_stream
        a = torch.ones(16, device="cuda")
        b = torch.empty_like(a)

        def quiet():
            torch.cuda.synchronize()
            comm.all_reduce(a.data_ptr(), b.data_ptr(), 16, 7, 0, st)
            torch.cuda.synchronize()

        moved = ctypes.c_size_t(0)
        out = {"rc": [], "moved": []}
        quiet()
        for pull, nbytes, wg in ((0, 64 << 20, 0), (1, 64 << 20, 0), (0, 3 << 20, 8), (1, 1, 5)):
            out["rc"].append(lib.nbxDebugLinkProbe(comm.handle, nbytes, pull, wg, st, ctypes.byref(moved)))
            out["moved"].append((nbytes, wg, int(moved.value)))
        quiet()
        out["bad"] = [lib.nbxDebugLinkProbe(comm.handle, 0, 0, 0, st, ctypes.byref(moved)),
                      lib.nbxDebugLinkProbe(comm.handle, 1 << 20, 0, -1, st, ctypes.byref(moved)),
                      lib.nbxDebugLinkProbe(comm.handle, 1 << 20, 0, 0, st, None)]
        count = 8 << 20   # 32 MiB fp32: the Simple protocol, through the staging the probe overwrote
        idx = torch.arange(count, dtype=torch.int32, device="cuda")
        x = ((idx * 7 + rank * 131) % 1000).to(torch.float32)
        y = torch.full_like(x, -1.0)
        comm.all_reduce(x.data_ptr(), y.data_ptr(), count, 7, 0, st)
        torch.cuda.synchronize()
        want = sum(((idx * 7 + r * 131) % 1000).to(torch.float32) for r in range(n))
        out["exact"] = bool(torch.equal(y, want))
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("n", [2, 3])
def test_multiprocess_link_probe(nbx, monkeypatch, n):
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "30")
    res = _run_ranks(nbx, n, _child_link_probe)
    for r in range(n):
        o = res[r]
        assert o["rc"] == [0, 0, 0, 0], o
        for nbytes, wg, moved in o["moved"]:
            assert moved >= nbytes and moved % (16 * (wg or 32)) == 0, (nbytes, wg, moved)
        assert o["bad"] == [4, 4, 4], o   # ncclInvalidArgument
        assert o["exact"], r


def _child_past_32_bits(uid_bytes, rank, n, q):
    """Counts past 2^32 through the multi-process communicator (size_t counts,
    nccl.h.in:315 / :331): a u8 sum AllReduce of 2^32 + 37 elements and a u8
    ReduceScatter whose send buffer holds n x (2^31 + 3) elements, on the
    Simple protocol, checked whole (uint8 adds wrap, as the reference's)."""
    try:
        import torch
        from tests.conftest import load_package
        nbx = load_package()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        st = torch.cuda.current_stream().cuda_stream

        def pattern(r, count):
            base = ((torch.arange(1 << 20, dtype=torch.int32, device="cuda") * 7 + 13 * r + 1) % 251).to(torch.uint8)
            return base.repeat(count // base.numel() + 1)[:count].contiguous()
        out = {}
        count = (1 << 32) + 37
        x = pattern(rank, count)
        y = torch.empty_like(x)
        comm.all_reduce(x.data_ptr(), y.data_ptr(), count, 1, 0, st)   # ncclUint8, ncclSum
        torch.cuda.synchronize()
        want = pattern(0, count)
        for r in range(1, n):
            want += pattern(r, count)
        out["allreduce"] = bool(torch.equal(y, want))
        del x, y, want
        torch.cuda.empty_cache()
        rc = (1 << 31) + 3
        x = pattern(rank, rc * n)
        y = torch.empty(rc, dtype=torch.uint8, device="cuda")
        comm.reduce_scatter(x.data_ptr(), y.data_ptr(), rc, 1, 0, st)
        torch.cuda.synchronize()
        want = pattern(0, rc * n)[rank * rc:(rank + 1) * rc].clone()
        for r in range(1, n):
            want += pattern(r, rc * n)[rank * rc:(rank + 1) * rc]
        out["reduce_scatter"] = bool(torch.equal(y, want))
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_multiprocess_counts_past_32_bits(nbx, monkeypatch):
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    res = _run_ranks(nbx, 2, _child_past_32_bits)
    for r in range(2):
        assert res[r] == {"allreduce": True, "reduce_scatter": True}, (r, res[r])


def _child_in_place(uid_bytes, rank, n, q):
    """In-place calls as the reference defines them (nccl.h.in:315-331):
    AllReduce with sendbuff == recvbuff, ReduceScatter with recvbuff ==
    sendbuff + rank * recvcount, Reduce with recvbuff == sendbuff on the root —
    at LL, LL128 (one- and two-shot) and Simple sizes, each compared bit for
    bit with the same call out of place (itself checked against the oracle by
    the suites above)."""
    try:
        import torch
        from tests.conftest import load_package
        nbx = load_package()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        st = torch.cuda.current_stream().cuda_stream
        g = torch.Generator(device="cuda").manual_seed(77 + rank)
        out = []
        for count in (1000, 100003, 2 * 1024 * 1024 + 5):   # LL, LL128 (two-shot above 256 KiB at n > 2), Simple
            for kind in ("allreduce", "reducescatter", "reduce"):
                total = count * n if kind == "reducescatter" else count
                x = torch.randn(total, generator=g, device="cuda")
                ref = torch.full((count,), -7.0, device="cuda")
                ip = x.clone()
                torch.cuda.synchronize()
                root = (n - 1) if kind == "reduce" else 0
                if kind == "allreduce":
                    comm.all_reduce(x.data_ptr(), ref.data_ptr(), count, 7, 0, st)
                    comm.all_reduce(ip.data_ptr(), ip.data_ptr(), count, 7, 0, st)
                    got = ip
                elif kind == "reducescatter":
                    comm.reduce_scatter(x.data_ptr(), ref.data_ptr(), count, 7, 0, st)
                    comm.reduce_scatter(ip.data_ptr(), ip[rank * count:].data_ptr(), count, 7, 0, st)
                    got = ip[rank * count:(rank + 1) * count]
                else:
                    comm.reduce(x.data_ptr(), ref.data_ptr() if rank == root else 0, count, 7, 0, root, st)
                    comm.reduce(ip.data_ptr(), ip.data_ptr() if rank == root else 0, count, 7, 0, root, st)
                    got = ip if rank == root else None
                torch.cuda.synchronize()
                same = True if got is None else bool(torch.equal(got, ref))
                untouched = True
                if kind == "reducescatter":   # the other blocks of the send buffer stay as they were
                    untouched = bool(torch.equal(ip[:rank * count], x[:rank * count]) and
                                     torch.equal(ip[(rank + 1) * count:], x[(rank + 1) * count:]))
                elif kind == "reduce" and rank != root:
                    untouched = bool(torch.equal(ip, x))
                out.append((count, kind, same, untouched))
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("n,algo", [(2, ""), (3, ""), (3, "Ring"), (4, "")])
def test_multiprocess_in_place(nbx, monkeypatch, n, algo):
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NCCL_ALGO", algo)
    res = _run_ranks(nbx, n, _child_in_place)
    for r in range(n):
        bad = [c for c in res[r] if not (c[2] and c[3])]
        assert not bad and len(res[r]) == 9, (r, bad)


# every type x every op through the multi-process communicator at each
# protocol's sizes (bytes per message; LL, LL128 one-shot, LL128 two-shot at
# n = 3, Simple), AllReduce throughout, ReduceScatter / Reduce for sum and max
EVERY_TYPE_BYTES = (4001, 100003, 600001, (3 << 20) + 5)


def _every_type_cases():
    cases = []
    for dtype in range(12):
        for b in EVERY_TYPE_BYTES:
            count = max(1, b // (8 if dtype in (4, 5, 8) else 4 if dtype in (2, 3, 7) else 2 if dtype in (6, 9) else 1))
            for op in range(5):
                cases.append(("ar", dtype, op, count))
            if b >= 100003:
                for op in (0, 2):
                    cases.append(("rs", dtype, op, max(1, count // 3)))
                    cases.append(("red", dtype, op, count))
    return cases


def _child_every_type(uid_bytes, rank, n, q):
    try:
        import torch
        from tests.conftest import load_package
        nbx = load_package()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        st = torch.cuda.current_stream().cuda_stream
        out = {}
        for i, (kind, dtype, op, count) in enumerate(_every_type_cases()):
            x = _ll_input(kind, dtype, count, n, rank).view(np.uint8)
            tx = torch.from_numpy(x.copy()).cuda()
            ty = torch.zeros(x.size // n if kind == "rs" else x.size, dtype=torch.uint8, device="cuda")
            if kind == "ar":
                comm.all_reduce(tx.data_ptr(), ty.data_ptr(), count, dtype, op, st)
            elif kind == "rs":
                comm.reduce_scatter(tx.data_ptr(), ty.data_ptr(), count, dtype, op, st)
            else:
                comm.reduce(tx.data_ptr(), ty.data_ptr(), count, dtype, op, _ll_root(i, n), st)
            torch.cuda.synchronize()
            out[i] = ty.cpu().numpy().copy()
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_multiprocess_every_type_and_op(nbx, oracle, monkeypatch):
    """All 12 types x sum / prod / max / min / avg as AllReduce, and
    ReduceScatter / Reduce for sum and max, through the multi-process
    communicator at LL, LL128 one-shot, LL128 two-shot and Simple sizes
    (3 ranks, odd byte counts), each bit-exact vs the oracle in the direct
    schedule's fold order."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    n = 3
    res = _run_ranks(nbx, n, _child_every_type)
    bad = []
    for i, (kind, dtype, op, count) in enumerate(_every_type_cases()):
        total = count * n if kind == "rs" else count
        xs = oracle.random_inputs(dtype, 8, total, seed=77 + dtype + count)[:n]   # = _ll_input, all ranks at once
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
        for r, e in exp.items():
            if not np.array_equal(res[r][i], np.ascontiguousarray(e).view(np.uint8)):
                bad.append((kind, dtype, op, count, r))
    assert not bad, bad[:10]


# user PreMulSum with a different scalar on every rank: the reference applies
# each rank's scalar to its own input only (prims_simple.h:269-270, :617-628),
# so the result is sum_r s_r * x_r. (dtype, count, kind); scalars per rank
PREMUL_CASES = [(7, 1000, "ar"), (7, 100003, "ar"), (7, 2 * 1024 * 1024 + 5, "ar"), (7, 100003, "rs"),
                (7, 2 * 1024 * 1024 + 5, "rs"), (7, 100003, "red"), (6, 40001, "ar"), (9, 700001, "ar"),
                (2, 100003, "ar"), (4, 5001, "red"), (10, 300001, "ar"), (8, 50001, "rs")]
PREMUL_FLOATS = (0.5, -1.25, 3.0, 0.75)
PREMUL_INTS = (3, -2, 5, 7)


def _premul_scalar(np_, dtype, r):
    from oracle import oracle
    st = oracle.NP_STORAGE[dtype]
    if dtype in (0, 1, 2, 3, 4, 5):
        return np_.array([PREMUL_INTS[r]]).astype(st)
    f = PREMUL_FLOATS[r]
    if dtype == 6:
        return np_.array([oracle.f32_to_f16(f)], dtype=st)
    if dtype == 9:
        return np_.array([oracle.f32_to_bf16(f)], dtype=st)
    if dtype == 10:
        return np_.array([oracle.f32_to_e4m3(f)], dtype=st)
    if dtype == 11:
        return np_.array([oracle.f32_to_e5m2(f)], dtype=st)
    return np_.array([f]).astype(st)


def _child_premul(uid_bytes, rank, n, q, device_scalar):
    try:
        import torch
        from tests.conftest import load_package
        nbx = load_package()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        st = torch.cuda.current_stream().cuda_stream
        out = {}
        for i, (dtype, count, kind) in enumerate(PREMUL_CASES):
            sc = _premul_scalar(np, dtype, rank)
            if device_scalar:
                dsc = torch.from_numpy(sc.view(np.uint8).copy()).cuda()
                op = comm.redop_create_premulsum(dsc.data_ptr(), dtype, nbx.ncclScalarResidence.ncclScalarDevice)
            else:
                op = comm.redop_create_premulsum(sc.ctypes.data, dtype)
            x = _ll_input(kind, dtype, count, n, rank).view(np.uint8)
            tx = torch.from_numpy(x.copy()).cuda()
            ty = torch.zeros(x.size // n if kind == "rs" else x.size, dtype=torch.uint8, device="cuda")
            root = 1 % n
            if kind == "ar":
                comm.all_reduce(tx.data_ptr(), ty.data_ptr(), count, dtype, op, st)
            elif kind == "rs":
                comm.reduce_scatter(tx.data_ptr(), ty.data_ptr(), count, dtype, op, st)
            else:
                comm.reduce(tx.data_ptr(), ty.data_ptr() if rank == root else 0, count, dtype, op, root, st)
            torch.cuda.synchronize()
            comm.redop_destroy(op)
            out[i] = ty.cpu().numpy().copy()
        # the same op inside a group next to an ordinary call (never batched with it)
        sc = _premul_scalar(np, 7, rank)
        op = comm.redop_create_premulsum(sc.ctypes.data, 7)
        x = _ll_input("ar", 7, 1000, n, rank)
        tx = torch.from_numpy(x.view(np.uint8).copy()).cuda()
        ty1 = torch.zeros(x.nbytes, dtype=torch.uint8, device="cuda")
        ty2 = torch.zeros(x.nbytes, dtype=torch.uint8, device="cuda")
        nbx.group_start()
        comm.all_reduce(tx.data_ptr(), ty1.data_ptr(), 1000, 7, 0, st)
        comm.all_reduce(tx.data_ptr(), ty2.data_ptr(), 1000, 7, op, st)
        nbx.group_end()
        torch.cuda.synchronize()
        comm.redop_destroy(op)
        out["group_sum"] = ty1.cpu().numpy().copy()
        out["group_premul"] = ty2.cpu().numpy().copy()
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def _premul_expected(oracle, kind, dtype, count, n, xs_by_rank):
    """sum over ranks of (x_r * s_r rounded to the type), folded in the
    direct schedule's order; expected per rank (Reduce: the root only)."""
    st = oracle.NP_STORAGE[dtype]
    eb = np.dtype(st).itemsize
    scaled = [oracle.reduce_multi([xs_by_rank[r]], dtype, 3, int(_premul_scalar(np, dtype, r).view(
        {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[eb])[0]), n_pre_op_srcs=1)[0] for r in range(n)]
    exp = {}
    if kind == "ar":
        full = np.empty(count, dtype=st)
        for c, (lo, hi) in enumerate(_blocks(count, eb, n)):
            if hi > lo:
                order = [(c + 1 + k) % n for k in range(n)]
                full[lo:hi] = oracle.reduce_multi([scaled[j][lo:hi] for j in order], dtype, 0)[0]
        exp = {r: full for r in range(n)}
    elif kind == "rs":
        for r in range(n):
            order = [(r + 1 + k) % n for k in range(n)]
            exp[r] = oracle.reduce_multi([scaled[j][r * count:(r + 1) * count] for j in order], dtype, 0)[0]
    else:
        root = 1 % n
        order = [(root + 1 + k) % n for k in range(n)]
        exp[root] = oracle.reduce_multi([scaled[j] for j in order], dtype, 0)[0]
    return exp


@pytest.mark.parametrize("n,device_scalar", [(2, False), (3, False), (3, True)])
def test_multiprocess_user_premulsum_per_rank_scalars(nbx, oracle, monkeypatch, n, device_scalar):
    """ncclRedOpCreatePreMulSum with a different scalar on every rank (host
    immediate or device-resident): sum_r s_r * x_r, as the reference computes
    it, at LL, LL128 and Simple sizes for AllReduce / ReduceScatter / Reduce
    and several types; inside a group it runs beside a plain Sum call."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    res = _run_ranks(nbx, n, _child_premul, device_scalar)
    bad = []
    for i, (dtype, count, kind) in enumerate(PREMUL_CASES):
        xs = [_ll_input(kind, dtype, count, n, r) for r in range(n)]
        for r, e in _premul_expected(oracle, kind, dtype, count, n, xs).items():
            if not np.array_equal(res[r][i], np.ascontiguousarray(e).view(np.uint8)):
                bad.append((kind, dtype, count, r))
    assert not bad, bad
    xs = [_ll_input("ar", 7, 1000, n, r) for r in range(n)]
    e = _premul_expected(oracle, "ar", 7, 1000, n, xs)[0]
    plain = np.empty(1000, np.float32)
    for c, (lo, hi) in enumerate(_blocks(1000, 4, n)):
        order = [(c + 1 + k) % n for k in range(n)]
        plain[lo:hi] = oracle.reduce_multi([xs[j][lo:hi] for j in order], 7, 0)[0]
    for r in range(n):
        mp_diag.check_equal(res[r]["group_premul"], e.view(np.uint8), ("group_premul", r))
        mp_diag.check_equal(res[r]["group_sum"], plain.view(np.uint8), ("group_sum", r))


def _child_split(uid_bytes, rank, n, q):
    """ncclCommSplit over a multi-process communicator: children ordered by
    key (ties by parent rank), NCCL_SPLIT_NOCOLOR gets NULL, every child works;
    ncclCommRegister / Deregister and ncclMemAlloc / Free round trips."""
    try:
        import ctypes

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        lib = nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        out = {}
        st = torch.cuda.current_stream().cuda_stream
        # split 1: color = rank % 2, key = n - rank (reverse order inside a color)
        child, rc = comm.split(rank % 2, n - rank)
        out["rc1"] = rc
        out["child1"] = (child.count(), child.user_rank())
        x = torch.full((1000,), float(rank + 1), device="cuda")
        y = torch.empty_like(x)
        child.all_reduce(x.data_ptr(), y.data_ptr(), 1000, 7, 0, st)
        torch.cuda.synchronize()
        out["sum1"] = float(y[0]) if torch.all(y == y[0]) else None
        # split 2: rank 1 opts out, the rest share color 5 with equal keys (parent order)
        child2, rc2 = comm.split(-1 if rank == 1 else 5, 0)
        out["rc2"] = rc2
        if child2 is not None:
            out["child2"] = (child2.count(), child2.user_rank())
            child2.all_reduce(x.data_ptr(), y.data_ptr(), 1000, 7, 0, st)
            torch.cuda.synchronize()
            out["sum2"] = float(y[0]) if torch.all(y == y[0]) else None
            child2.destroy()
        else:
            out["child2"] = None
        # registration and ncclMemAlloc
        h = comm.register(x.data_ptr(), x.numel() * 4)
        comm.deregister(h)
        p = ctypes.c_void_p()
        assert lib.ncclMemAlloc(ctypes.byref(p), 1 << 20) == 0 and p.value
        assert lib.ncclMemFree(p) == 0
        child.destroy()
        comm.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_multiprocess_comm_split(nbx, monkeypatch):
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    n = 4
    res = _run_ranks(nbx, n, _child_split)
    for r in range(n):
        same = [p for p in range(n) if p % 2 == r % 2]
        order = sorted(same, key=lambda p: (n - p, p))
        assert res[r]["rc1"] == 0
        assert res[r]["child1"] == (len(same), order.index(r)), (r, res[r])
        assert res[r]["sum1"] == float(sum(p + 1 for p in same)), (r, res[r])
        if r == 1:
            assert res[r]["child2"] is None
        else:
            members = [p for p in range(n) if p != 1]
            assert res[r]["child2"] == (len(members), members.index(r)), (r, res[r])
            assert res[r]["sum2"] == float(sum(p + 1 for p in members)), (r, res[r])


def _child_knobs(uid_bytes, rank, n, q, env, cfg=None):
    """The reference's own knobs (NCCL_BUFFSIZE, NCCL_LL_BUFFSIZE,
    NCCL_LL128_BUFFSIZE, NCCL_MAX/MIN_NCHANNELS) as the communicator applies
    them, then exact AllReduces at an LL, an LL128 and a Simple size. `env`:
    per-rank environment set before ncclCommInitRank (values may differ by
    rank: {name: [value of rank 0, value of rank 1, ...]})."""
    try:
        import ctypes
        import os

        import torch
        from tests.conftest import load_package
        for k, vals in env.items():
            os.environ[k] = vals[rank]
        nbx = load_package()
        lib = nbx.load_library()
        torch.cuda.set_device(0)
        uid = nbx.ncclUniqueId.from_buffer_copy(uid_bytes)
        try:
            if cfg is None:
                comm = nbx.Communicator.init_rank(n, uid, rank)
            else:   # ncclConfig_t fields (minCTAs / maxCTAs ...)
                comm, rc = nbx.Communicator.init_rank_config(n, uid, rank, **cfg)
        except nbx.NcclError as e:
            q.put((rank, "ok", {"init": int(e.code)}))
            return
        vals = (ctypes.c_int64 * 10)()
        got = lib.nbxDebugCommSettings(comm.handle, vals, 10)
        out = {"init": 0, "settings": list(vals)[:got]}
        st = torch.cuda.current_stream().cuda_stream
        for cnt in (2048, 131072, 1 << 20):   # 8 KiB (LL), 512 KiB (LL128), 4 MiB (Simple) of fp32
            x = torch.remainder(torch.arange(cnt, device="cuda", dtype=torch.float32) * 3 + rank, 101)
            y = torch.full((cnt,), -1.0, device="cuda")
            comm.all_reduce(x.data_ptr(), y.data_ptr(), cnt, 7, 0, st)
            torch.cuda.synchronize()
            want = sum(torch.remainder(torch.arange(cnt, device="cuda", dtype=torch.float32) * 3 + r, 101)
                       for r in range(n))
            out[cnt] = bool(torch.equal(y, want))
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("buffsize,slice_want", [("65536", 32768), ("4194304", 65536)])
def test_multiprocess_reference_knobs(nbx, monkeypatch, buffsize, slice_want):
    """NCCL_BUFFSIZE 64 KiB -> 32 KiB Simple slices (2 slots), while the
    reference's own 4 MiB default, set explicitly, leaves the 64 KiB slice (only
    smaller buffers are honoured: ADVICE r4, 1 MiB slices would be 4 GiB of
    staging at 8 ranks); NCCL_LL_BUFFSIZE 64 KiB -> LL up to 32 KiB,
    NCCL_LL128_BUFFSIZE 1 MiB -> LL128 up to 768 KiB, NCCL_MAX_NCHANNELS 16 ->
    every grid capped at 16 workgroups; results exact."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    for k in ("NBX_SIMPLE_SLICE_BYTES", "NBX_SIMPLE_MAX_GRID", "NBX_LL_MAX_BYTES", "NBX_LL128_MAX_BYTES"):
        monkeypatch.delenv(k, raising=False)
    n = 2
    env = {"NCCL_BUFFSIZE": [buffsize] * n, "NCCL_LL_BUFFSIZE": ["65536"] * n,
           "NCCL_LL128_BUFFSIZE": ["1048576"] * n, "NCCL_MAX_NCHANNELS": ["16"] * n}
    res = _run_ranks(nbx, n, _child_knobs, env)
    for r in range(n):
        assert res[r]["init"] == 0
        ll, l128, slice_, slots, grid, llcap, l128cap, batch = res[r]["settings"][:8]
        assert (ll, l128, slice_, slots, grid) == (32768, 786432, slice_want, 2, 16), res[r]["settings"]
        assert llcap <= 16 and l128cap <= 16 and batch == 1
        assert res[r]["settings"][9] == 0   # plan checks off by default
        assert all(res[r][c] for c in (2048, 131072, 1 << 20)), res[r]


@pytest.mark.parametrize("cfg,env,grid", [({"maxCTAs": 8}, {}, 8), ({"minCTAs": 16, "maxCTAs": 64}, {}, 64),
                                          ({"maxCTAs": 64}, {"NCCL_MAX_CTAS": ["4", "4"]}, 4),
                                          ({"maxCTAs": 100}, {"NCCL_MAX_NCHANNELS": ["12", "12"]}, 12)])
def test_multiprocess_config_ctas(nbx, monkeypatch, cfg, env, grid):
    """ncclConfig_t minCTAs / maxCTAs (a CTA / channel is a workgroup here,
    connect.cc:418-422: min(NCCL_MAX_NCHANNELS, maxCTAs) and at least
    max(NCCL_MIN_NCHANNELS, minCTAs)), NCCL_MAX_CTAS overriding the config
    (envConfigOverride, init.cc:1460-1463): the Simple grid and the LL / LL128
    caps follow; results exact."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    for k in ("NBX_SIMPLE_MAX_GRID", "NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_MIN_CTAS", "NCCL_MAX_CTAS"):
        monkeypatch.delenv(k, raising=False)
    res = _run_ranks(nbx, 2, _child_knobs, env, cfg)
    for r in range(2):
        assert res[r]["init"] == 0, res[r]
        ll, l128, slice_, slots, g, llcap, l128cap = res[r]["settings"][:7]
        assert g == grid and llcap <= grid and l128cap <= grid, res[r]["settings"]
        assert all(res[r][c] for c in (2048, 131072, 1 << 20)), res[r]


@pytest.mark.parametrize("name", ["NCCL_CHECK_POINTERS", "NBX_CHECK_PLANS"])
def test_multiprocess_plan_checks_on_exact(nbx, monkeypatch, name):
    """The reference's argument-checking knob (or NBX_CHECK_PLANS) turns the
    plan words / slice headers on; LL, LL128 and Simple results stay exact."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.delenv("NBX_CHECK_PLANS", raising=False)
    res = _run_ranks(nbx, 2, _child_knobs, {name: ["1", "1"]})
    for r in range(2):
        assert res[r]["init"] == 0 and res[r]["settings"][9] == 1, res[r]
        assert all(res[r][c] for c in (2048, 131072, 1 << 20)), res[r]


def test_multiprocess_nbx_override_wins(nbx, monkeypatch):
    """An NBX_* setting set next to the reference knob it maps wins."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    n = 2
    env = {"NCCL_BUFFSIZE": ["262144"] * n, "NBX_SIMPLE_SLICE_BYTES": ["16384"] * n,
           "NCCL_MIN_NCHANNELS": ["8"] * n, "NCCL_MAX_NCHANNELS": ["4"] * n, "NBX_SIMPLE_MAX_GRID": ["6"] * n}
    res = _run_ranks(nbx, n, _child_knobs, env)
    for r in range(n):
        assert res[r]["settings"][2] == 16384 and res[r]["settings"][4] == 6, res[r]["settings"]
        assert all(res[r][c] for c in (2048, 131072, 1 << 20)), res[r]


@pytest.mark.parametrize("name,vals", [("NCCL_BUFFSIZE", ["65536", "32768"]), ("NBX_GROUP_BATCH", ["1", "0"]),
                                       ("NCCL_LL_BUFFSIZE", ["65536", "32768"]), ("NBX_CHECK_PLANS", ["1", "0"])])
def test_multiprocess_settings_must_agree(nbx, monkeypatch, name, vals):
    """Settings that decide a call's protocol, grid, staging layout or launch
    cut must be equal on every rank: ncclCommInitRank fails with
    ncclInvalidUsage on every rank instead of the ranks' kernels disagreeing."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    for k in ("NBX_SIMPLE_SLICE_BYTES", "NBX_LL_MAX_BYTES", "NBX_GROUP_BATCH", "NBX_CHECK_PLANS"):
        monkeypatch.delenv(k, raising=False)
    res = _run_ranks(nbx, 2, _child_knobs, {name: vals})
    for r in range(2):
        assert res[r]["init"] == int(nbx.ncclResult.ncclInvalidUsage), (r, res[r])


@pytest.mark.parametrize("buf", [0, 1, 2, 3])
def test_multiprocess_ipc_mapping_repair(nbx, monkeypatch, buf):
    """A connection buffer whose peers' mappings fail the creation-time check
    is re-exported and re-mapped, and the communicator then works exactly
    (NBX_IPC_VERIFY_FAIL: rank 1 reports buffer `buf` — LL, LL128, staging,
    flags — wrong in the first check round)."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NBX_IPC_VERIFY_FAIL", f"1:{buf}")
    n = 3
    res = _run_ranks(nbx, n, _child_knobs, {})
    for r in range(n):
        assert res[r]["init"] == 0
        assert res[r]["settings"][8] == 1, res[r]["settings"]   # one buffer re-exported, seen by every rank
        assert all(res[r][c] for c in (2048, 131072, 1 << 20)), res[r]


def _child_comm_churn(uid_list, rank, n, q):
    """Communicators created and destroyed back to back (the pattern that
    makes the runtime hand out wrong IPC mappings now and then,
    scripts/probe_ipc_export.py): every one must come up with verified
    mappings and run an LL, an LL128 and a Simple AllReduce exactly."""
    try:
        import ctypes

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        lib = nbx.load_library()
        torch.cuda.set_device(0)
        st = torch.cuda.current_stream().cuda_stream
        out = {"repairs": 0, "exact": 0, "wrong": []}
        keep = None
        for i, ub in enumerate(uid_list):
            comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(ub), rank)
            vals = (ctypes.c_int64 * 9)()
            assert lib.nbxDebugCommSettings(comm.handle, vals, 9) == 9
            out["repairs"] += vals[8]
            for cnt in (1000 + i, 70001 + 7 * i, (1 << 20) + 3 * i):   # LL, LL128, Simple
                x = torch.remainder(torch.arange(cnt, device="cuda", dtype=torch.float32) * 3 + rank + i, 89)
                y = torch.full((cnt,), -1.0, device="cuda")
                comm.all_reduce(x.data_ptr(), y.data_ptr(), cnt, 7, 0, st)
                torch.cuda.synchronize()
                want = sum(torch.remainder(torch.arange(cnt, device="cuda", dtype=torch.float32) * 3 + r + i, 89)
                           for r in range(n))
                if torch.equal(y, want):
                    out["exact"] += 1
                else:
                    out["wrong"].append((i, cnt))
            # like ncclCommSplit: now and then the previous communicator outlives the next one's creation
            if keep is not None:
                keep.destroy()
                keep = None
            if i % 3 == 1:
                keep = comm
            else:
                comm.destroy()
        if keep is not None:
            keep.destroy()
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_multiprocess_comm_churn_verified_mappings(nbx, monkeypatch):
    """40 communicators of 3 ranks in a row: every collective exact; the
    creation-time check re-exports whatever mapping the runtime got wrong."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    n, k = 3, 40
    uids = [bytes(nbx.get_unique_id()) for _ in range(k)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_child_comm_churn, args=(uids, r, n, q), daemon=True) for r in range(n)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(n):
            rank, status, payload = q.get(timeout=280)
            assert status == "ok", f"rank {rank}:\n{payload}"
            res[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    for r in range(n):
        assert res[r]["wrong"] == [] and res[r]["exact"] == 3 * k, (r, res[r])
    print("re-exported connection buffers over", k, "communicators:", [res[r]["repairs"] for r in range(n)])


def _child_abort_pending_init(uid_bytes, rank, q, evq):
    """Rank 0 initialises non-blocking with the LL128 creation probe forced on,
    rank 1 skips the probe (NBX_LL128_SELFTEST_ITERS=0), so rank 0's
    background initialisation ends up in a probe kernel waiting for lines rank 1
    never sends; ncclCommAbort must end that device wait (the communicator's
    abort word is set before the init thread is joined) instead of waiting out
    NBX_TIMEOUT_SEC."""
    try:
        import os
        import time

        import torch
        from tests.conftest import load_package
        os.environ["NBX_LL128_SELFTEST_ITERS"] = "8" if rank == 0 else "0"
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        uid = nbx.ncclUniqueId.from_buffer_copy(uid_bytes)
        if rank == 1:
            comm = nbx.Communicator.init_rank(2, uid, 1)
            evq.get(timeout=240)   # rank 0 has aborted
            comm.destroy()
            q.put((rank, "ok", None))
            return
        comm, rc = nbx.Communicator.init_rank_config(2, uid, 0, blocking=0)
        assert rc == int(nbx.ncclResult.ncclInProgress), rc
        time.sleep(6.0)   # connection setup done; the probe's first kernel is waiting on rank 1
        pending = comm.async_error()
        t0 = time.perf_counter()
        comm.abort()
        dt = time.perf_counter() - t0
        evq.put("done")
        q.put((rank, "ok", {"pending": pending, "abort_s": dt}))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_multiprocess_abort_ends_pending_init_device_wait(nbx, monkeypatch):
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "120")
    ctx = mp.get_context("spawn")
    uid = nbx.get_unique_id()
    q, evq = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_child_abort_pending_init, args=(bytes(uid), r, q, evq), daemon=True)
             for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(2):
            rank, status, payload = q.get(timeout=280)
            assert status == "ok", f"rank {rank}:\n{payload}"
            res[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    assert res[0]["pending"] == int(nbx.ncclResult.ncclInProgress), res[0]   # still initialising
    assert res[0]["abort_s"] < 20, res[0]                                      # not the 120 s timeout


def _child_plan_mismatch(uid_bytes, rank, n, q, case, cnt=300000):
    """Ranks whose launches are cut from different plans: every Simple slice
    carries its producer's plan signature, every LL / LL128 source stamps its
    plan word, so the consumer fails the launch (ncclRemoteError, the check
    named "... different plan ...") instead of folding misplaced data or
    timing out. case "count": the ranks pass different counts; "op": the same
    count, rank 1 reduces with max (its lines do arrive); "group": rank 0's
    group reads what its previous call wrote (cut into two launches), rank 1's
    calls are independent (one launch)."""
    try:
        import ctypes

        import torch
        from tests.conftest import load_package
        nbx = load_package()
        lib = nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        st = torch.cuda.current_stream().cuda_stream
        a = torch.ones(cnt + 8, device="cuda")
        b = torch.zeros(cnt + 8, device="cuda")
        c = torch.zeros(cnt + 8, device="cuda")
        d = torch.ones(cnt + 8, device="cuda")
        if case == "count":
            comm.all_reduce(a.data_ptr(), b.data_ptr(), cnt + (3 if rank == 1 else 0), 7, 0, st)
        elif case == "op":
            comm.all_reduce(a.data_ptr(), b.data_ptr(), cnt, 7, 2 if rank == 1 else 0, st)
        else:
            nbx.group_start()
            comm.all_reduce(a.data_ptr(), b.data_ptr(), cnt, 7, 0, st)
            comm.all_reduce((b if rank == 0 else d).data_ptr(), c.data_ptr(), cnt, 7, 0, st)
            nbx.group_end()
        torch.cuda.synchronize()
        err = comm.async_error()
        msg = (lib.ncclGetLastError(None) or b"").decode(errors="replace")
        comm.abort()
        q.put((rank, "ok", {"err": err, "msg": msg}))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("case", ["count", "group"])
def test_multiprocess_simple_plan_mismatch_fails_loudly(nbx, monkeypatch, case):
    monkeypatch.setenv("NCCL_CHECK_POINTERS", "1")   # turns the plan checks on (NBX_CHECK_PLANS default)
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "5")
    monkeypatch.setenv("NCCL_PROTO", "Simple")
    monkeypatch.setenv("NCCL_DEBUG", "WARN")
    res = _run_ranks(nbx, 2, _child_plan_mismatch, case)
    remote = int(nbx.ncclResult.ncclRemoteError)
    assert all(res[r]["err"] == remote for r in range(2)), res
    assert any("different plan" in res[r]["msg"] for r in range(2)), res


# LL (4 KiB), LL128 one-shot (80 KB) and two-shot (1.2 MB): a peer that runs the
# same call with another plan is named by its plan word well before the 5 s
# timeout (a timeout would read "timed out", not "different plan")
@pytest.mark.parametrize("proto,cnt,case", [("LL", 1000, "count"), ("LL", 1000, "op"), ("LL", 1000, "group"),
                                            ("LL128", 20000, "count"), ("LL128", 20000, "op"),
                                            ("LL128", 300000, "count"), ("LL128", 300000, "op")])
def test_multiprocess_ll_plan_mismatch_fails_loudly(nbx, monkeypatch, proto, cnt, case):
    monkeypatch.setenv("NBX_CHECK_PLANS", "1")
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "5")
    monkeypatch.setenv("NCCL_PROTO", proto)
    monkeypatch.setenv("NCCL_DEBUG", "WARN")
    res = _run_ranks(nbx, 2, _child_plan_mismatch, case, cnt)
    remote = int(nbx.ncclResult.ncclRemoteError)
    assert all(res[r]["err"] == remote for r in range(2)), res
    assert all("different plan" in res[r]["msg"] for r in range(2)), res


# ---------------------------------------------------------------------------
# Simple slice checksums (NBX_CHECK_SLICES): every staging slice carries a hash
# of its elements that the consumer recomputes from what it read.

SLICE_CASES = [  # (kind, dtype, op, count, byte offset): pack and element paths, fold and copy, every kind
    ("ar", 7, 0, 1100000, 0), ("ar", 2, 2, 1000003, 0), ("ar", 7, 0, 300000, 4), ("ar", 6, 4, 700001, 2),
    ("ar", 9, 0, 650000, 0), ("ar", 0, 3, 2500001, 1), ("ar", 8, 1, 200001, 0), ("ar", 11, 0, 1300001, 0),
    ("rs", 7, 4, 1048577, 0), ("rs", 4, 2, 150000, 8), ("red", 7, 0, 300001, 0), ("red", 2, 3, 500000, 4),
]


def _child_slices(uid_bytes, rank, n, q, iters=2):
    try:
        import torch
        from tests.conftest import load_package
        nbx = load_package()
        lib = nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        settings = mp_diag.comm_settings(nbx, comm)
        st = torch.cuda.current_stream().cuda_stream
        out = {}
        for it in range(iters):
            keep = []
            for i, (kind, dtype, op, count, shift) in enumerate(SLICE_CASES):
                x = _ll_input(kind, dtype, count, n, rank).view(np.uint8)
                tx = torch.zeros(x.size + 16, dtype=torch.uint8, device="cuda")
                tx[shift:shift + x.size] = torch.from_numpy(x.copy()).cuda()
                out_bytes = x.size // n if kind == "rs" else x.size
                ty = torch.zeros(out_bytes + 16, dtype=torch.uint8, device="cuda")
                sp, rp = tx.data_ptr() + shift, ty.data_ptr() + shift
                if kind == "ar":
                    comm.all_reduce(sp, rp, count, dtype, op, st)
                elif kind == "rs":
                    comm.reduce_scatter(sp, rp, count, dtype, op, st)
                else:
                    comm.reduce(sp, rp, count, dtype, op, _ll_root(i, n), st)
                keep.append((i, ty, tx, shift, out_bytes))   # no host sync between calls
            torch.cuda.synchronize()
            for i, ty, _tx, shift, nb in keep:
                out[(it, i)] = ty[shift:shift + nb].cpu().numpy().copy()
        err = comm.async_error()
        msg = (lib.ncclGetLastError(None) or b"").decode(errors="replace")
        comm.abort() if err else comm.destroy()
        q.put((rank, "ok", {"out": out, "err": err, "msg": msg, "settings": settings}))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("n,algo", [(3, ""), (4, "Ring"), (8, "")])
def test_multiprocess_simple_slice_checksums(nbx, oracle, monkeypatch, n, algo):
    """NBX_CHECK_SLICES=1 on the Simple direct and ring schedules: every
    producer's stamped sum equals what its consumers recompute (no false
    alarm on any path — 16-B packs, element tails, misaligned buffers, every
    element width, fold and copy hops), and the outputs stay bit-exact."""
    monkeypatch.setenv("NBX_CHECK_SLICES", "1")
    monkeypatch.setenv("NCCL_PROTO", "Simple")
    monkeypatch.setenv("NCCL_ALGO", algo)
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    res = _run_ranks(nbx, n, _child_slices)
    for r in range(n):
        assert res[r]["err"] == 0, (r, res[r]["msg"])
        assert res[r]["settings"].get("checkSlices") == 1
    failures = []
    for i, (kind, dtype, op, count, shift) in enumerate(SLICE_CASES):
        xs = [_ll_input(kind, dtype, count, n, r) for r in range(n)]
        devop, arg = oracle.host_to_dev_redop(op, dtype, n)
        st = oracle.NP_STORAGE[dtype]
        eb = np.dtype(st).itemsize
        kw = dict(n_pre_op_srcs=n, post_op=devop == 4)
        root = _ll_root(i, n)
        if algo == "Ring" and kind != "ar":
            continue   # ring ReduceScatter / Reduce fold in NCCL's chain order: test_multiprocess_ring_fifo_*
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
            order = [(root + 1 + k) % n for k in range(n)]
            exp[root] = oracle.reduce_multi([xs[j] for j in order], dtype, devop, arg, **kw)[0]
        for it in range(2):
            for r, e in exp.items():
                got = res[r]["out"][(it, i)]
                if not np.array_equal(got, np.ascontiguousarray(e).view(np.uint8)):
                    failures.append((f"slice-check case {i} {SLICE_CASES[i]} iteration {it}", kind, dtype, op, count,
                                     r, got, xs, res[r]["settings"], root))
    mp_diag.raise_collective_failures(oracle, failures, n, what=f"NBX_CHECK_SLICES=1 NCCL_ALGO={algo or 'direct'}: ")


@pytest.mark.parametrize("algo", ["", "Ring"])
def test_multiprocess_simple_slice_checksum_catches_a_wrong_slice(nbx, monkeypatch, algo):
    """The negative case: rank 1's workgroup 0 stamps a wrong sum
    (NBX_DEBUG_SLICE_FAULT=1), as a slice whose bytes changed between the
    producer's stores and the consumer's loads would read. Its consumers fail
    the call loudly — ncclRemoteError, the check named with the peer, the slot
    use and both sums — instead of returning a result nobody verified."""
    monkeypatch.setenv("NBX_CHECK_SLICES", "1")
    monkeypatch.setenv("NBX_DEBUG_SLICE_FAULT", "1")
    monkeypatch.setenv("NCCL_PROTO", "Simple")
    monkeypatch.setenv("NCCL_ALGO", algo)
    monkeypatch.setenv("NCCL_DEBUG", "WARN")
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "10")
    res = _run_ranks(nbx, 3, _child_slices, 1)
    remote = int(nbx.ncclResult.ncclRemoteError)
    flagged = [r for r in range(3) if res[r]["err"] == remote]
    assert flagged, {r: (res[r]["err"], res[r]["msg"]) for r in range(3)}
    assert any("Simple slice checksum" in res[r]["msg"] and "from peer 1" in res[r]["msg"] for r in flagged), \
        {r: res[r]["msg"] for r in range(3)}


def _child_replay(uid_bytes, rank, n, q, case_ids, iters):
    """LL_CASES[case_ids] back to back (no host sync inside an iteration), the
    send and recv buffers inside 4 KiB 0xA5 canaries checked after every
    iteration; returns every output."""
    try:
        import torch
        from tests.conftest import load_package
        nbx = load_package()
        lib = nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        settings = mp_diag.comm_settings(nbx, comm)
        st = torch.cuda.current_stream().cuda_stream
        G = 4096
        out, canary = {}, []
        for it in range(iters):
            keep = []
            for i in case_ids:
                kind, dtype, op, count, shift = LL_CASES[i]
                x = _ll_input(kind, dtype, count, n, rank).view(np.uint8)
                tx = torch.full((x.size + 16 + 2 * G,), 0xA5, dtype=torch.uint8, device="cuda")
                tx[G:G + x.size + 16] = 0
                tx[G + shift:G + shift + x.size] = torch.from_numpy(x.copy()).cuda()
                nb = x.size // n if kind == "rs" else x.size
                ty = torch.full((nb + 16 + 2 * G,), 0xA5, dtype=torch.uint8, device="cuda")
                ty[G:G + nb + 16] = 0
                sp, rp = tx.data_ptr() + G + shift, ty.data_ptr() + G + shift
                if kind == "ar":
                    comm.all_reduce(sp, rp, count, dtype, op, st)
                elif kind == "rs":
                    comm.reduce_scatter(sp, rp, count, dtype, op, st)
                else:
                    comm.reduce(sp, rp, count, dtype, op, _ll_root(i, n), st)
                keep.append((i, tx, ty, shift, nb))
            torch.cuda.synchronize()
            for i, tx, ty, shift, nb in keep:
                out[(it, i)] = ty[G + shift:G + shift + nb].cpu().numpy().copy()
                for name, t in (("send", tx), ("recv", ty)):
                    if not (bool((t[:G] == 0xA5).all()) and bool((t[t.numel() - G:] == 0xA5).all())):
                        canary.append((it, i, name))
        err = comm.async_error()
        assert err == 0, (err, (lib.ncclGetLastError(None) or b"").decode(errors="replace"))
        comm.destroy()
        q.put((rank, "ok", {"out": out, "canary": canary, "settings": settings}))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_multiprocess_gputest_r05_replay_cases_32_37(nbx, oracle, monkeypatch):
    """the calls around GPUTEST_r05's red record — LL128
    two-shot cases 32-34, Simple case 35 (misaligned fp32), Simple case 36
    (int32 max, 1,000,003 elements: the wrong one), Simple case 37 (fp64) —
    at 8 ranks sharing the GPU, back to back, 12 iterations; every output of
    every rank bit-exact vs the oracle (described if not), and no byte outside
    a call's own buffers written."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "60")
    monkeypatch.setenv("NBX_LL128_MAX_GRID", "16")
    n, cases, iters = 8, list(range(32, 38)), 12
    res = _run_ranks(nbx, n, _child_replay, cases, iters)
    assert not any(res[r]["canary"] for r in range(n)), {r: res[r]["canary"][:4] for r in range(n)}
    failures = []
    for i in cases:
        kind, dtype, op, count, shift = LL_CASES[i]
        xs = [_ll_input(kind, dtype, count, n, r) for r in range(n)]
        devop, arg = oracle.host_to_dev_redop(op, dtype, n)
        st = oracle.NP_STORAGE[dtype]
        eb = np.dtype(st).itemsize
        kw = dict(n_pre_op_srcs=n, post_op=devop == 4)
        assert kind == "ar"
        full = np.empty(count, dtype=st)
        for c, (lo, hi) in enumerate(_blocks(count, eb, n)):
            if hi > lo:
                order = [(c + 1 + k) % n for k in range(n)]
                full[lo:hi] = oracle.reduce_multi([xs[j][lo:hi] for j in order], dtype, devop, arg, **kw)[0]
        want = np.ascontiguousarray(full).view(np.uint8)
        for it in range(iters):
            for r in range(n):
                got = res[r]["out"][(it, i)]
                if not np.array_equal(got, want):
                    failures.append((f"replay case {i} {LL_CASES[i]} iteration {it}", kind, dtype, op, count, r,
                                     got, xs, res[r]["settings"], None))
    mp_diag.raise_collective_failures(oracle, failures, n, what="GPUTEST_r05 replay: ")
