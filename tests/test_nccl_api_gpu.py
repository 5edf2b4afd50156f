"""GPU tests of the NCCL API layer (nccl_api.cc and the comm_*.cc units) over the reduction core.

World size 1 follows taskAppend -> ncclLaunchOneRank (enqueue.cc:1564-1566,
onerank.cu:48-79): PreMulSum runs the kernel, every other op is a copy.
The in-process clique (ncclCommInitAll) is exercised with several ranks that
share the one GPU of the test box; its documented fold order for block r is
ranks r+1, r+2, ..., r (NCCL's ring reduce-scatter order).
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

F32, F16, I32, BF16, F64, I8, U64 = 7, 6, 2, 9, 8, 0, 5


def t_of(torch, a):
    return torch.from_numpy(a.view(np.uint8).copy()).cuda()


def np_of(t, dtype):
    return t.cpu().numpy().view(dtype)


@pytest.fixture
def comm1(nbx, torch_gpu):
    c = nbx.Communicator.init_rank(1, nbx.get_unique_id(), 0)
    yield c
    c.destroy()


def test_comm_queries(nbx, comm1):
    assert comm1.count() == 1 and comm1.user_rank() == 0 and comm1.device() == 0
    assert comm1.async_error() == 0


@pytest.mark.parametrize("dtype", [I8, I32, U64, F16, F32, F64, BF16, 10])
@pytest.mark.parametrize("op", [0, 1, 2, 3, 4])
def test_one_rank_allreduce_semantics(nbx, oracle, torch_gpu, comm1, dtype, op):
    torch = torch_gpu
    st = torch.cuda.current_stream().cuda_stream
    x = oracle.random_inputs(dtype, 1, 5003, seed=dtype * 7 + op)[0]
    tx = t_of(torch, x)
    ty = torch.zeros_like(tx)
    comm1.all_reduce(tx.data_ptr(), ty.data_ptr(), x.size, dtype, op, st)
    torch.cuda.synchronize()
    devop, arg = oracle.host_to_dev_redop(op, dtype, 1)
    if devop == 3:   # PreMulSum (float Avg): kernel with pre-op on the one source
        exp = oracle.reduce_multi([x], dtype, devop, arg, n_pre_op_srcs=1, post_op=True)[0]
    else:            # copy (onerank.cu:50-55)
        exp = x
    assert np.array_equal(np_of(ty, x.dtype).view(np.uint8), exp.view(np.uint8))


def test_one_rank_in_place_and_reduce_scatter_and_reduce(nbx, oracle, torch_gpu, comm1):
    torch = torch_gpu
    st = torch.cuda.current_stream().cuda_stream
    x = oracle.random_inputs(F32, 1, 4096, seed=3)[0]
    tx = t_of(torch, x)
    comm1.all_reduce(tx.data_ptr(), tx.data_ptr(), x.size, F32, 0, st)       # in place: no-op
    ty = torch.zeros_like(tx)
    comm1.reduce_scatter(tx.data_ptr(), ty.data_ptr(), x.size, F32, 0, st)
    tz = torch.zeros_like(tx)
    comm1.reduce(tx.data_ptr(), tz.data_ptr(), x.size, F32, 2, 0, st)
    torch.cuda.synchronize()
    for t in (tx, ty, tz):
        assert np.array_equal(np_of(t, np.float32), x)
    with pytest.raises(nbx.NcclError) as e:
        comm1.reduce(tx.data_ptr(), tz.data_ptr(), x.size, F32, 0, 1, st)   # root out of range
    assert e.value.code == nbx.ncclResult.ncclInvalidArgument
    with pytest.raises(nbx.NcclError):
        comm1.all_reduce(tx.data_ptr(), ty.data_ptr(), x.size, 12, 0, st)    # bad type
    with pytest.raises(nbx.NcclError):
        comm1.all_reduce(tx.data_ptr(), ty.data_ptr(), x.size, F32, 77, st)  # unknown op


def test_user_premulsum_host_and_device_scalar(nbx, oracle, torch_gpu, comm1):
    torch = torch_gpu
    st = torch.cuda.current_stream().cuda_stream
    x = oracle.random_inputs(F32, 1, 8191, seed=11)[0]
    tx = t_of(torch, x)
    ty = torch.zeros_like(tx)
    s = ctypes.c_float(0.3)
    op = comm1.redop_create_premulsum(ctypes.addressof(s), F32, nbx.ncclScalarResidence.ncclScalarHostImmediate)
    assert op >= 5
    s.value = 9.0   # host-immediate: captured at creation
    comm1.all_reduce(tx.data_ptr(), ty.data_ptr(), x.size, F32, op, st)
    torch.cuda.synchronize()
    exp = oracle.reduce_multi([x], F32, 3, int(np.float32(0.3).view(np.uint32)), 1, True)[0]
    assert np.array_equal(np_of(ty, np.float32), exp)
    # device-resident scalar: dereferenced while the kernel runs
    ds = torch.tensor([0.0], dtype=torch.float32, device="cuda")
    op2 = comm1.redop_create_premulsum(ds.data_ptr(), F32, nbx.ncclScalarResidence.ncclScalarDevice)
    ds.fill_(-1.75)
    comm1.all_reduce(tx.data_ptr(), ty.data_ptr(), x.size, F32, op2, st)
    torch.cuda.synchronize()
    exp2 = oracle.reduce_multi([x], F32, 3, int(np.float32(-1.75).view(np.uint32)), 1, True)[0]
    assert np.array_equal(np_of(ty, np.float32), exp2)
    with pytest.raises(nbx.NcclError):   # op created for F32 used with F16
        comm1.all_reduce(tx.data_ptr(), ty.data_ptr(), 16, F16, op, st)
    comm1.redop_destroy(op)
    comm1.redop_destroy(op2)
    with pytest.raises(nbx.NcclError):
        comm1.all_reduce(tx.data_ptr(), ty.data_ptr(), x.size, F32, op, st)
    with pytest.raises(nbx.NcclError):
        comm1.redop_destroy(op)


def _ring_order_reduce(oracle, xs, dtype, devop, arg, post, nranks, block_of, root=None):
    """Oracle for the clique: block r folded in rank order r+1, ..., r
    (AllReduce / ReduceScatter), or root+1, ..., root for every block (Reduce)."""
    st = oracle.NP_STORAGE[dtype]
    count = xs[0].size
    out = np.empty(count, dtype=st)
    for r in range(nranks):
        lo, hi = block_of(r)
        if hi <= lo:
            continue
        first = (r if root is None else root) + 1
        order = [(first + k) % nranks for k in range(nranks)]
        out[lo:hi] = oracle.reduce_multi([xs[j][lo:hi] for j in order], dtype, devop, arg,
                                         n_pre_op_srcs=nranks, post_op=post)[0]
    return out


def _blocks(count, eb, n):
    epp = 16 // eb
    per = -(-count // n)
    per = -(-per // epp) * epp
    return lambda b: (min(count, per * b), min(count, per * b + per))


@pytest.mark.parametrize("nranks", [2, 3, 4])
@pytest.mark.parametrize("dtype,op", [(F32, 0), (F32, 4), (F16, 0), (BF16, 4), (I32, 4), (I32, 2), (F64, 3)])
def test_clique_allreduce_shared_device(nbx, oracle, torch_gpu, nranks, dtype, op):
    torch = torch_gpu
    comms = nbx.Communicator.init_all([0] * nranks)
    try:
        assert [c.user_rank() for c in comms] == list(range(nranks))
        count = 30011
        xs = oracle.random_inputs(dtype, nranks, count, seed=nranks * 100 + dtype)
        txs = [t_of(torch, x) for x in xs]
        tys = [torch.zeros_like(t) for t in txs]
        streams = [torch.cuda.Stream() for _ in range(nranks)]
        torch.cuda.synchronize()
        nbx.group_start()
        for r in range(nranks):
            comms[r].all_reduce(txs[r].data_ptr(), tys[r].data_ptr(), count, dtype, op, streams[r].cuda_stream)
        nbx.group_end()
        torch.cuda.synchronize()
        devop, arg = oracle.host_to_dev_redop(op, dtype, nranks)
        eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
        exp = _ring_order_reduce(oracle, xs, dtype, devop, arg, devop == 4, nranks, _blocks(count, eb, nranks))
        for r in range(nranks):
            got = np_of(tys[r], exp.dtype)
            assert np.array_equal(got.view(np.uint8), exp.view(np.uint8)), f"rank {r}"
    finally:
        for c in comms:
            c.destroy()


def test_clique_counts_past_32_bits(nbx, torch_gpu):
    """Counts past 2^32 through ncclCommInitAll (2 ranks on the one GPU: the
    event-ordered direct fold): u8 sum AllReduce of 2^32 + 37 elements and a
    ReduceScatter of recvcount 2^31 + 3, checked whole (u8 adds wrap)."""
    torch = torch_gpu
    comms = nbx.Communicator.init_all([0, 0])

    def pattern(r, count):
        base = ((torch.arange(1 << 20, dtype=torch.int32, device="cuda") * 5 + 29 * r + 3) % 253).to(torch.uint8)
        return base.repeat(count // base.numel() + 1)[:count].contiguous()
    try:
        count = (1 << 32) + 37
        xs = [pattern(r, count) for r in range(2)]
        ys = [torch.empty_like(x) for x in xs]
        streams = [torch.cuda.Stream() for _ in range(2)]
        torch.cuda.synchronize()
        nbx.group_start()
        for r in range(2):
            comms[r].all_reduce(xs[r].data_ptr(), ys[r].data_ptr(), count, 1, 0, streams[r].cuda_stream)
        nbx.group_end()
        torch.cuda.synchronize()
        want = xs[0] + xs[1]
        assert torch.equal(ys[0], want) and torch.equal(ys[1], want)
        del xs, ys, want
        torch.cuda.empty_cache()
        rc = (1 << 31) + 3
        xs = [pattern(r, 2 * rc) for r in range(2)]
        ys = [torch.empty(rc, dtype=torch.uint8, device="cuda") for _ in range(2)]
        torch.cuda.synchronize()
        nbx.group_start()
        for r in range(2):
            comms[r].reduce_scatter(xs[r].data_ptr(), ys[r].data_ptr(), rc, 1, 0, streams[r].cuda_stream)
        nbx.group_end()
        torch.cuda.synchronize()
        for r in range(2):
            assert torch.equal(ys[r], xs[0][r * rc:(r + 1) * rc] + xs[1][r * rc:(r + 1) * rc]), r
    finally:
        for c in comms:
            c.destroy()


def test_clique_user_premulsum_alternating_streams_no_sync(nbx, oracle, torch_gpu):
    """back-to-back per-rank PreMulSum AllReduces on a clique,
    alternating each rank's stream between two streams with no host sync. Each
    call's pre-pass rewrites the rank's one scratch buffer, which the peers'
    folds of the previous call (on the other stream) read in place: the pre-pass
    must wait for them (preScratchFree). 64 MiB per rank keeps the calls on the
    fold path; every output is checked bit-exact."""
    torch = torch_gpu
    nranks, count, calls = 3, 16 << 20, 4
    scal = (0.5, -1.25, 3.0)
    comms = nbx.Communicator.init_all([0] * nranks)
    streams = [[torch.cuda.Stream() for _ in range(2)] for _ in range(nranks)]
    try:
        hs = [np.array([s_], np.float32).view(np.uint32) for s_ in scal]
        ops = [comms[r].redop_create_premulsum(hs[r].ctypes.data, F32) for r in range(nranks)]
        ins, outs = [], []
        for k in range(calls):
            xs = oracle.random_inputs(F32, nranks, count, seed=300 + k)
            ins.append((xs, [t_of(torch, x) for x in xs]))
            outs.append([torch.zeros(count * 4, dtype=torch.uint8, device="cuda") for _ in range(nranks)])
        torch.cuda.synchronize()
        for k in range(calls):
            nbx.group_start()
            for r in range(nranks):
                comms[r].all_reduce(ins[k][1][r].data_ptr(), outs[k][r].data_ptr(), count, F32, ops[r],
                                    streams[r][k % 2].cuda_stream)
            nbx.group_end()
        torch.cuda.synchronize()
        for r in range(nranks):
            comms[r].redop_destroy(ops[r])
        for k in range(calls):
            xs = ins[k][0]
            scaled = [oracle.reduce_multi([xs[r]], F32, 3, int(hs[r][0]), n_pre_op_srcs=1)[0] for r in range(nranks)]
            exp = _ring_order_reduce(oracle, scaled, F32, 0, 0, False, nranks, _blocks(count, 4, nranks))
            for r in range(nranks):
                assert np.array_equal(outs[k][r].cpu().numpy(), np.ascontiguousarray(exp).view(np.uint8)), (k, r)
    finally:
        for c in comms:
            c.destroy()


def test_clique_user_premulsum_per_rank_scalars(nbx, oracle, torch_gpu):
    """A 3-rank clique with a different PreMulSum scalar per rank: sum_r s_r x_r
    (the reference's per-rank pre-op), AllReduce / ReduceScatter / Reduce on
    the fold path, f32 and bf16."""
    torch = torch_gpu
    nranks = 3
    scal = (0.5, -1.25, 3.0)
    comms = nbx.Communicator.init_all([0] * nranks)
    streams = [torch.cuda.Stream() for _ in range(nranks)]
    try:
        for dtype in (F32, BF16):
            st_ = oracle.NP_STORAGE[dtype]
            eb = np.dtype(st_).itemsize
            bits = [np.array([s_], np.float32).view(np.uint32)[0] if dtype == F32 else oracle.f32_to_bf16(s_)
                    for s_ in scal]
            hs = [np.array([b], dtype=np.uint32 if dtype == F32 else np.uint16) for b in bits]
            for kind in ("ar", "rs", "red"):
                count = 50003
                total = count * nranks if kind == "rs" else count
                xs = oracle.random_inputs(dtype, nranks, total, seed=61 + dtype)
                txs = [t_of(torch, x) for x in xs]
                outs = [torch.zeros(count * eb, dtype=torch.uint8, device="cuda") for _ in range(nranks)]
                ops = [comms[r].redop_create_premulsum(hs[r].ctypes.data, dtype) for r in range(nranks)]
                torch.cuda.synchronize()
                nbx.group_start()
                for r in range(nranks):
                    sp, rp, s_ = txs[r].data_ptr(), outs[r].data_ptr(), streams[r].cuda_stream
                    if kind == "ar":
                        comms[r].all_reduce(sp, rp, count, dtype, ops[r], s_)
                    elif kind == "rs":
                        comms[r].reduce_scatter(sp, rp, count, dtype, ops[r], s_)
                    else:
                        comms[r].reduce(sp, rp if r == 2 else 0, count, dtype, ops[r], 2, s_)
                nbx.group_end()
                torch.cuda.synchronize()
                for r in range(nranks):
                    comms[r].redop_destroy(ops[r])
                scaled = [oracle.reduce_multi([xs[r]], dtype, 3, int(bits[r]), n_pre_op_srcs=1)[0]
                          for r in range(nranks)]
                if kind == "ar":
                    exp = _ring_order_reduce(oracle, scaled, dtype, 0, 0, False, nranks, _blocks(count, eb, nranks))
                    want = {r: exp for r in range(nranks)}
                elif kind == "rs":
                    exp = _ring_order_reduce(oracle, scaled, dtype, 0, 0, False, nranks,
                                             lambda b: (b * count, (b + 1) * count))
                    want = {r: exp[r * count:(r + 1) * count] for r in range(nranks)}
                else:
                    want = {2: _ring_order_reduce(oracle, scaled, dtype, 0, 0, False, nranks,
                                                  _blocks(count, eb, nranks), root=2)}
                for r, e in want.items():
                    assert np.array_equal(outs[r].cpu().numpy(), np.ascontiguousarray(e).view(np.uint8)), \
                        (dtype, kind, r)
    finally:
        for c in comms:
            c.destroy()


def test_clique_every_type_and_op(nbx, oracle, torch_gpu):
    """Every type x sum / prod / max / min / avg as a 3-rank clique AllReduce
    (odd count, the event-ordered direct fold), and ReduceScatter / Reduce
    for sum and max, bit-exact vs the oracle in the clique's fold orders."""
    torch = torch_gpu
    nranks = 3
    comms = nbx.Communicator.init_all([0] * nranks)
    streams = [torch.cuda.Stream() for _ in range(nranks)]
    bad = []
    try:
        for dtype in range(12):
            eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
            count = 60001 // eb + 3
            for op in range(5):
                kinds = ("ar", "rs", "red") if op in (0, 2) else ("ar",)
                for kind in kinds:
                    total = count * nranks if kind == "rs" else count
                    xs = oracle.random_inputs(dtype, nranks, total, seed=300 + 7 * dtype + op)
                    txs = [t_of(torch, x) for x in xs]
                    outs = [torch.zeros(count * eb, dtype=torch.uint8, device="cuda") for _ in range(nranks)]
                    torch.cuda.synchronize()
                    nbx.group_start()
                    for r in range(nranks):
                        sp, rp, s_ = txs[r].data_ptr(), outs[r].data_ptr(), streams[r].cuda_stream
                        if kind == "ar":
                            comms[r].all_reduce(sp, rp, count, dtype, op, s_)
                        elif kind == "rs":
                            comms[r].reduce_scatter(sp, rp, count, dtype, op, s_)
                        else:
                            comms[r].reduce(sp, rp if r == 2 else 0, count, dtype, op, 2, s_)
                    nbx.group_end()
                    torch.cuda.synchronize()
                    devop, arg = oracle.host_to_dev_redop(op, dtype, nranks)
                    if kind == "ar":
                        exp = _ring_order_reduce(oracle, xs, dtype, devop, arg, devop == 4, nranks,
                                                 _blocks(count, eb, nranks))
                        want = {r: exp for r in range(nranks)}
                    elif kind == "rs":
                        exp = _ring_order_reduce(oracle, xs, dtype, devop, arg, devop == 4, nranks,
                                                 lambda b: (b * count, (b + 1) * count))
                        want = {r: exp[r * count:(r + 1) * count] for r in range(nranks)}
                    else:
                        want = {2: _ring_order_reduce(oracle, xs, dtype, devop, arg, devop == 4, nranks,
                                                      _blocks(count, eb, nranks), root=2)}
                    for r, e in want.items():
                        if not np.array_equal(outs[r].cpu().numpy(), np.ascontiguousarray(e).view(np.uint8)):
                            bad.append((kind, dtype, op, r))
    finally:
        for c in comms:
            c.destroy()
    assert not bad, bad[:10]


@pytest.mark.parametrize("nranks", [2, 3])
def test_clique_reduce_scatter_and_reduce(nbx, oracle, torch_gpu, nranks):
    torch = torch_gpu
    comms = nbx.Communicator.init_all([0] * nranks)
    try:
        recvcount = 10007
        xs = oracle.random_inputs(F32, nranks, recvcount * nranks, seed=5)
        txs = [t_of(torch, x) for x in xs]
        # in place for rank 1: recvbuff == sendbuff + rank * recvcount
        outs = [torch.zeros(recvcount * 4, dtype=torch.uint8, device="cuda") for _ in range(nranks)]
        rptr = [o.data_ptr() for o in outs]
        rptr[1] = txs[1].data_ptr() + 1 * recvcount * 4
        nbx.group_start()
        for r in range(nranks):
            comms[r].reduce_scatter(txs[r].data_ptr(), rptr[r], recvcount, F32, 0, 0)
        nbx.group_end()
        torch.cuda.synchronize()
        exp = _ring_order_reduce(oracle, xs, F32, 0, 0, False, nranks,
                                 lambda b: (b * recvcount, (b + 1) * recvcount))
        for r in range(nranks):
            got = np_of(outs[r], np.float32) if r != 1 else \
                np_of(txs[1], np.float32)[recvcount:2 * recvcount]
            assert np.array_equal(got, exp[r * recvcount:(r + 1) * recvcount]), f"rank {r}"
        # ncclReduce to root 1 (ranks write their reduced block into the root's buffer)
        count = 20000
        ys = oracle.random_inputs(I32, nranks, count, seed=9)
        tys = [t_of(torch, y) for y in ys]
        root_out = torch.zeros(count * 4, dtype=torch.uint8, device="cuda")
        nbx.group_start()
        for r in range(nranks):
            comms[r].reduce(tys[r].data_ptr(), root_out.data_ptr() if r == 1 else 0, count, I32, 4, 1, 0)
        nbx.group_end()
        torch.cuda.synchronize()
        exp = _ring_order_reduce(oracle, ys, I32, 4, nranks, True, nranks, _blocks(count, 4, nranks), root=1)
        assert np.array_equal(np_of(root_out, np.int32), exp)
        # float Reduce: the chain order toward the root matters bitwise
        zs = oracle.random_inputs(F32, nranks, count, seed=19)
        tzs = [t_of(torch, z) for z in zs]
        root_f = torch.zeros(count * 4, dtype=torch.uint8, device="cuda")
        nbx.group_start()
        for r in range(nranks):
            comms[r].reduce(tzs[r].data_ptr(), root_f.data_ptr() if r == 0 else 0, count, F32, 0, 0, 0)
        nbx.group_end()
        torch.cuda.synchronize()
        exp = _ring_order_reduce(oracle, zs, F32, 0, 0, False, nranks, _blocks(count, 4, nranks), root=0)
        assert np.array_equal(np_of(root_f, np.float32), exp)
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("nranks", [9, 12])
def test_clique_in_place_past_8_ranks(nbx, oracle, torch_gpu, nranks):
    """In-place AllReduce (recv == send), ReduceScatter (recv == send +
    rank * recvcount) and Reduce (root's recv == send) with more than 8 ranks:
    the fold takes several passes and the rank's own block — its output — is
    read last, so the partial goes through scratch memory. Checked
    against the oracle in the schedule's fold order."""
    torch = torch_gpu
    comms = nbx.Communicator.init_all([0] * nranks)
    try:
        count = 20011
        xs = oracle.random_inputs(F32, nranks, count, seed=900 + nranks)
        txs = [t_of(torch, x) for x in xs]
        nbx.group_start()
        for r in range(nranks):
            comms[r].all_reduce(txs[r].data_ptr(), txs[r].data_ptr(), count, F32, 0, 0)
        nbx.group_end()
        torch.cuda.synchronize()
        exp = _ring_order_reduce(oracle, xs, F32, 0, 0, False, nranks, _blocks(count, 4, nranks))
        for r in range(nranks):
            assert np.array_equal(np_of(txs[r], np.float32), exp), f"allreduce rank {r}"
        rc = 3001
        ys = oracle.random_inputs(I32, nranks, rc * nranks, seed=910 + nranks)
        tys = [t_of(torch, y) for y in ys]
        nbx.group_start()
        for r in range(nranks):
            comms[r].reduce_scatter(tys[r].data_ptr(), tys[r].data_ptr() + r * rc * 4, rc, I32, 4, 0)
        nbx.group_end()
        torch.cuda.synchronize()
        devop, arg = oracle.host_to_dev_redop(4, I32, nranks)
        exp = _ring_order_reduce(oracle, ys, I32, devop, arg, True, nranks, lambda b: (b * rc, (b + 1) * rc))
        for r in range(nranks):
            got = np_of(tys[r], np.int32)[r * rc:(r + 1) * rc]
            assert np.array_equal(got, exp[r * rc:(r + 1) * rc]), f"reduce_scatter rank {r}"
        zs = oracle.random_inputs(F32, nranks, count, seed=920 + nranks)
        tzs = [t_of(torch, z) for z in zs]
        root = nranks - 1
        nbx.group_start()
        for r in range(nranks):
            comms[r].reduce(tzs[r].data_ptr(), tzs[r].data_ptr() if r == root else 0, count, F32, 0, root, 0)
        nbx.group_end()
        torch.cuda.synchronize()
        exp = _ring_order_reduce(oracle, zs, F32, 0, 0, False, nranks, _blocks(count, 4, nranks), root=root)
        assert np.array_equal(np_of(tzs[root], np.float32), exp)
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("nranks", [2, 3, 9])
def test_clique_grouped_collectives_batched(nbx, oracle, torch_gpu, nranks):
    """A group of independent collectives runs as one batched exchange (one
    enter/leave, one nbxReduceMultiBatch per rank and (datatype, op)); a
    collective that reads an earlier one's output, a change of stream, and
    AllReduce past 8 ranks (gather step) split the batch — results identical
    to running them one by one."""
    torch = torch_gpu
    comms = nbx.Communicator.init_all([0] * nranks)
    try:
        specs = [(F32, 0, 5000), (F32, 0, 77), (F16, 0, 30000), (BF16, 4, 12345), (I32, 2, 999), (I32, 4, 4096),
                 (F32, 0, 1), (F64, 3, 2500)]
        cases = []
        nbx.group_start()
        for k, (dt, op, count) in enumerate(specs):
            xs = oracle.random_inputs(dt, nranks, count, seed=1000 + 10 * nranks + k)
            txs = [t_of(torch, x) for x in xs]
            tys = [torch.zeros_like(t) for t in txs]
            for r in range(nranks):
                comms[r].all_reduce(txs[r].data_ptr(), tys[r].data_ptr(), count, dt, op, 0)
            cases.append((dt, op, count, xs, tys, txs))   # inputs stay alive until the group ends
        # a reduce-scatter in the same group
        rc = 3001
        rxs = oracle.random_inputs(F32, nranks, rc * nranks, seed=77)
        trx = [t_of(torch, x) for x in rxs]
        rout = [torch.zeros(rc, dtype=torch.float32, device="cuda") for _ in range(nranks)]
        for r in range(nranks):
            comms[r].reduce_scatter(trx[r].data_ptr(), rout[r].data_ptr(), rc, F32, 0, 0)
        # dependent: AllReduce of the first collective's output (must see it complete)
        dt0, op0, c0, _, tys0, _ = cases[0]
        dep = [torch.zeros_like(t) for t in tys0]
        for r in range(nranks):
            comms[r].all_reduce(tys0[r].data_ptr(), dep[r].data_ptr(), c0, dt0, op0, 0)
        nbx.group_end()
        torch.cuda.synchronize()
        for dt, op, count, xs, tys, _ in cases:
            devop, arg = oracle.host_to_dev_redop(op, dt, nranks)
            eb = np.dtype(oracle.NP_STORAGE[dt]).itemsize
            exp = _ring_order_reduce(oracle, xs, dt, devop, arg, devop == 4, nranks, _blocks(count, eb, nranks))
            for r in range(nranks):
                got = np_of(tys[r], exp.dtype)
                assert np.array_equal(got.view(np.uint8), exp.view(np.uint8)), f"dt {dt} op {op} n {count} rank {r}"
        exp_rs = _ring_order_reduce(oracle, rxs, F32, 0, 0, False, nranks, lambda b: (b * rc, (b + 1) * rc))
        for r in range(nranks):
            assert np.array_equal(np_of(rout[r], np.float32), exp_rs[r * rc:(r + 1) * rc]), f"rs rank {r}"
        first = [np_of(t, np.float32) for t in tys0]
        exp_dep = _ring_order_reduce(oracle, first, F32, 0, 0, False, nranks, _blocks(c0, 4, nranks))
        for r in range(nranks):
            assert np.array_equal(np_of(dep[r], np.float32), exp_dep), f"dependent rank {r}"
    finally:
        for c in comms:
            c.destroy()


def test_graph_capture_one_rank_kernel(nbx, oracle, torch_gpu, comm1):
    """The launch path does no allocation or sync, so it captures into a graph."""
    torch = torch_gpu
    x = oracle.random_inputs(F16, 1, 65536, seed=2)[0]
    tx = t_of(torch, x)
    ty = torch.zeros_like(tx)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    h = np.float16(0.25).view(np.uint16)
    hs = ctypes.c_uint16(int(h))
    op = comm1.redop_create_premulsum(ctypes.addressof(hs), F16, nbx.ncclScalarResidence.ncclScalarHostImmediate)
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            comm1.all_reduce(tx.data_ptr(), ty.data_ptr(), x.size, F16, op, torch.cuda.current_stream().cuda_stream)
    g.replay()
    torch.cuda.synchronize()
    exp = oracle.reduce_multi([x], F16, 3, int(h), 1, True)[0]
    assert np.array_equal(np_of(ty, np.uint16), exp)
    comm1.redop_destroy(op)


def test_nonblocking_init_abort_is_prompt(nbx, monkeypatch):
    """ncclCommAbort on a non-blocking communicator whose initialisation is
    still waiting for its peers (rank 1 never comes): the background thread's
    bootstrap waits end at the abort flag within ~0.1 s, long before the
    bootstrap timeout, and the communicator is freed."""
    import time
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "60")
    uid = nbx.get_unique_id()
    comm, rc = nbx.Communicator.init_rank_config(2, uid, 0, blocking=0)
    assert rc == int(nbx.ncclResult.ncclInProgress)
    time.sleep(0.3)
    assert comm.async_error() == int(nbx.ncclResult.ncclInProgress)
    t0 = time.monotonic()
    comm.abort()
    assert time.monotonic() - t0 < 5.0
