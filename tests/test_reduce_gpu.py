"""GPU parity of the hot path (nbxReduceMulti, the reduceCopy replacement)
against the CPU oracle — bit-exact for every type (integers, and floats folded
in the same order with correctly-rounded ops; NaN compared as NaN).

Inputs are seeded (oracle.random_inputs); sizes are small enough for the
oracle to finish in seconds, plus the BASELINE full-size configs through the
multithreaded oracle.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ALL_TYPES = list(range(12))
FLOAT_TYPES = {6, 7, 8, 9, 10, 11}


def devops_for(dtype):
    ops = [0, 1, 2, 3]
    if dtype not in FLOAT_TYPES:
        ops.append(4)
    return ops


def op_arg(oracle, dtype, devop, rng):
    """A representative scalarArg for the device op."""
    if devop == 2:   # MinMax: alternate min / max encodings from hostToDevRedOp
        return oracle.host_to_dev_redop(2 if rng.integers(2) else 3, dtype, 1)[1]
    if devop == 3:   # PreMulSum: the Avg scalar for 3 ranks (inexact in most types)
        return oracle.host_to_dev_redop(4, dtype, 3)[1] if dtype in FLOAT_TYPES else int(rng.integers(1, 1 << 16))
    if devop == 4:
        return 3
    return 0


class Dev:
    """Device staging: a torch uint8 buffer per array, optional byte offset."""

    def __init__(self, torch):
        self.torch = torch
        self.keep = []

    def upload(self, a: np.ndarray, offset: int = 0) -> int:
        t = self.torch.empty(a.nbytes + offset + 64, dtype=self.torch.uint8, device="cuda")
        if a.nbytes:
            t[offset:offset + a.nbytes].copy_(self.torch.from_numpy(a.view(np.uint8).copy()))
        self.keep.append(t)
        return t.data_ptr() + offset

    def alloc(self, nbytes: int, offset: int = 0):
        t = self.torch.full((nbytes + offset + 64,), 0xA5, dtype=self.torch.uint8, device="cuda")
        self.keep.append(t)
        return t, t.data_ptr() + offset

    @staticmethod
    def download(t, offset, nbytes, dtype):
        return t[offset:offset + nbytes].cpu().numpy().view(dtype)


def assert_same(got, exp, dtype):
    assert got.shape == exp.shape
    if dtype in FLOAT_TYPES:
        if dtype in (7, 8):
            gn, en = np.isnan(got), np.isnan(exp)
        else:
            dec = {6: _dec16, 9: _decbf16, 10: _dec_e4m3, 11: _dec_e5m2}[dtype]
            gn, en = dec(got), dec(exp)
        assert np.array_equal(gn, en), f"NaN mismatch at {np.flatnonzero(gn != en)[:8]}"
        keep = ~en
        ut = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[got.itemsize]
        bad = np.flatnonzero(got.view(ut)[keep] != exp.view(ut)[keep])
        assert bad.size == 0, f"{bad.size} mismatches, first at {np.flatnonzero(keep)[bad[:8]]}: " \
                              f"got {got.view(ut)[keep][bad[:4]]} exp {exp.view(ut)[keep][bad[:4]]}"
    else:
        bad = np.flatnonzero(got != exp)
        assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:8]}: got {got[bad[:4]]} exp {exp[bad[:4]]}"


def _dec16(a):
    return ((a & 0x7C00) == 0x7C00) & ((a & 0x3FF) != 0)


def _decbf16(a):
    return ((a & 0x7F80) == 0x7F80) & ((a & 0x7F) != 0)


def _dec_e4m3(a):
    return (a & 0x7F) == 0x7F


def _dec_e5m2(a):
    return ((a & 0x7C) == 0x7C) & ((a & 0x03) != 0)


def run_case(nbx, oracle, torch, srcs, dtype, devop, arg, npre=0, post=False, ndst=1, src_off=None, dst_off=None,
             arg_on_device=False):
    dev = Dev(torch)
    count = srcs[0].size
    st = oracle.NP_STORAGE[dtype]
    eb = np.dtype(st).itemsize
    src_off = src_off or [0] * len(srcs)
    dst_off = dst_off or [0] * ndst
    sp = [dev.upload(s, o) for s, o in zip(srcs, src_off)]
    outs = [dev.alloc(count * eb, o) for o in dst_off]
    op = nbx.DevRedOpFull()
    op.op = devop
    if arg_on_device:
        scal = dev.upload(np.array([arg], dtype=np.uint64).view(np.uint8)[:eb].copy())
        op.scalarArgIsPtr = 1
        op.scalarArg = scal
    else:
        op.scalarArg = arg
    stream = torch.cuda.current_stream().cuda_stream
    nbx.reduce_multi([p for _, p in outs], sp, count, dtype, op, npre, post, stream)
    torch.cuda.synchronize()
    exp = oracle.reduce_multi(srcs, dtype, devop, arg, npre, post, n_dsts=1, threads=8)[0]
    for (t, _), o in zip(outs, dst_off):
        got = Dev.download(t, o, count * eb, st)
        assert_same(got, exp, dtype)
        # bytes around the destination untouched (no overrun)
        tail = t[o + count * eb:].cpu().numpy()
        assert (tail == 0xA5).all() and (t[:o].cpu().numpy() == 0xA5).all()
    return exp


@pytest.mark.parametrize("dtype", ALL_TYPES)
@pytest.mark.parametrize("nsrc", [1, 2, 3, 8])
def test_all_types_ops(nbx, oracle, torch_gpu, dtype, nsrc):
    rng = np.random.default_rng(100 + dtype * 10 + nsrc)
    for devop in devops_for(dtype):
        srcs = oracle.random_inputs(dtype, nsrc, 4099, seed=int(rng.integers(1 << 30)), specials=True)
        arg = op_arg(oracle, dtype, devop, rng)
        npre = int(rng.integers(0, nsrc + 1)) if devop == 3 else 0
        run_case(nbx, oracle, torch_gpu, srcs, dtype, devop, arg, npre=npre, post=(devop == 4))


@pytest.mark.parametrize("count", [0, 1, 3, 15, 16, 17, 255, 4095, 4096, 65537, 1 << 20])
@pytest.mark.parametrize("dtype", [1, 6, 7, 8])
def test_edge_sizes(nbx, oracle, torch_gpu, dtype, count):
    for nsrc in (2, 8):
        srcs = oracle.random_inputs(dtype, nsrc, count, seed=7 + count)
        if count == 0:
            dev = Dev(torch_gpu)
            op = nbx.DevRedOpFull()
            rc = nbx.reduce_multi_raw([dev.upload(np.zeros(4, np.uint8))], [dev.upload(np.zeros(4, np.uint8))] * nsrc,
                                      0, dtype, op)
            assert rc == 0
            continue
        run_case(nbx, oracle, torch_gpu, srcs, dtype, 0, 0)


@pytest.mark.parametrize("dtype", [0, 6, 7, 9, 4])
def test_shared_misalignment(nbx, oracle, torch_gpu, dtype):
    """All pointers share one misalignment modulo 16 -> head peeling + fast body."""
    eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
    for off in range(eb, 16, eb):
        srcs = oracle.random_inputs(dtype, 3, 10001, seed=off)
        run_case(nbx, oracle, torch_gpu, srcs, dtype, 0, 0, src_off=[off] * 3, dst_off=[off])


@pytest.mark.parametrize("dtype", [1, 6, 7, 8])
def test_mixed_misalignment(nbx, oracle, torch_gpu, dtype):
    """Different alignments modulo 16: sources realigned against one destination
    alignment (kReduceShifted), or destinations of different alignments (element
    kernel, common_kernel.h:229-238)."""
    eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
    srcs = oracle.random_inputs(dtype, 4, 12345, seed=3)
    run_case(nbx, oracle, torch_gpu, srcs, dtype, 0, 0, src_off=[0, eb, 0, 2 * eb % 16], dst_off=[eb % 16])
    run_case(nbx, oracle, torch_gpu, srcs, dtype, 2, 0, ndst=2, src_off=[eb % 16, 0, 0, 0], dst_off=[0, eb % 16])


@pytest.mark.parametrize("dtype", [0, 6, 7, 4, 10, 9])
@pytest.mark.parametrize("count", [1, 7, 100, 4097, 70001])
def test_realigned_sources(nbx, oracle, torch_gpu, dtype, count):
    """Sources at alignments that differ from the destinations' (kReduceShifted:
    16-B packs on the destination side, every source realigned in registers by
    its own byte offset): every offset an element size allows, 1-8 sources,
    1-3 destinations sharing one alignment, heads and tails, every op."""
    eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
    offs = list(range(0, 16, eb))
    rng = np.random.default_rng(count * 16 + dtype)
    for devop in devops_for(dtype):
        nsrc = 1 + (devop * 3 + count) % 8
        srcs = oracle.random_inputs(dtype, nsrc, count, seed=int(rng.integers(1 << 20)))
        src_off = [offs[(k * 5 + devop + 1) % len(offs)] for k in range(nsrc)]
        dst_o = offs[(devop + 2) % len(offs)]
        ndst = 1 + devop % 3
        arg = op_arg(oracle, dtype, devop, rng)
        run_case(nbx, oracle, torch_gpu, srcs, dtype, devop, arg, npre=min(2, nsrc) if devop == 3 else 0,
                 post=devop == 4, ndst=ndst, src_off=src_off, dst_off=[dst_o] * ndst)


@pytest.mark.parametrize("dtype,nsrc,count", [(7, 8, 3_000_001), (7, 4, 2_097_155), (6, 5, 4_194_309),
                                              (9, 3, 1_048_583), (10, 8, 8_388_617)])
def test_realigned_sources_grid_stride(nbx, oracle, torch_gpu, dtype, nsrc, count):
    """Realigned sources at sizes where the waves stride past the grid (more
    tiles than one pass of the LDS-DMA kernel covers): stage reuse, the
    lane-0 extra pack of every tile, ragged last tile."""
    eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
    srcs = oracle.random_inputs(dtype, nsrc, count, seed=nsrc * 7 + dtype)
    src_off = [(k * 3 * eb) % 16 for k in range(nsrc)]
    run_case(nbx, oracle, torch_gpu, srcs, dtype, 0, 0, src_off=src_off, dst_off=[eb % 16])


@pytest.mark.parametrize("dtype,nsrc,count", [(7, 8, 3_000_001), (7, 4, 2_097_155), (6, 5, 4_194_309),
                                              (9, 3, 1_048_583), (10, 8, 8_388_617), (7, 2, 1_500_007),
                                              (7, 8, 70_001), (7, 3, 5_003)])
def test_realigned_sources_dynamic_schedule(nbx, oracle, torch_gpu, dynamic_tiles_always, dtype, nsrc, count):
    """The realigning kernel's dynamic schedule (class counters, forced for
    every launch here): many tiles per wave, and few (classes with fewer tiles
    than waves, where every fetch is terminal)."""
    eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
    srcs = oracle.random_inputs(dtype, nsrc, count, seed=nsrc * 11 + dtype + count % 97)
    src_off = [(k * 3 * eb + eb) % 16 for k in range(nsrc)]
    run_case(nbx, oracle, torch_gpu, srcs, dtype, 0, 0, src_off=src_off, dst_off=[0])


def test_realigned_dynamic_back_to_back_and_streams(nbx, oracle, torch_gpu, dynamic_tiles_always):
    """Class counters reset themselves on each class's last fetch: launches
    of different sizes issued back to back on one stream (no host sync), and
    on two streams at once, all come out exact — a counter left non-zero would
    make the next launch skip tiles (its outputs keep the sentinel)."""
    torch = torch_gpu
    dtype, nsrc = 7, 8
    lib = nbx.load_library()
    cases = []
    for k, n in enumerate([2_000_003, 9_001, 1_048_577, 3_000_017, 50_021]):
        srcs = oracle.random_inputs(dtype, nsrc, n, seed=1200 + k)
        exp = oracle.reduce_multi(srcs, dtype, 0, threads=8)[0]
        # sources one element into their buffers, destination aligned: realigned
        ts = [torch.from_numpy(np.concatenate([np.zeros(1, np.float32), x])).cuda() for x in srcs]
        out = torch.full((n,), -7.0, dtype=torch.float32, device="cuda")
        cases.append((ts, out, exp, n))
    op = nbx.DevRedOpFull()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()

    def call(ts, out, n, st):
        sp = (ctypes.c_void_p * nsrc)(*[t.data_ptr() + 4 for t in ts])
        dp = (ctypes.c_void_p * 1)(out.data_ptr())
        assert lib.nbxReduceMulti(dp, 1, sp, nsrc, ctypes.c_size_t(n), dtype, op, 0, 0, ctypes.c_void_p(st)) == 0

    for rep in range(3):
        for k, (ts, out, exp, n) in enumerate(cases):   # back to back, alternating streams by case
            call(ts, out, n, streams[(k + rep) % 2].cuda_stream)
        torch.cuda.synchronize()
        for ts, out, exp, n in cases:
            assert_same(out.cpu().numpy(), exp, dtype)
            out.fill_(-7.0)
        torch.cuda.synchronize()


def _hip():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    lib.hipFree.argtypes = [ctypes.c_void_p]
    lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return lib


@pytest.mark.parametrize("dtype,nsrc", [(7, 2), (7, 5), (7, 8), (10, 3), (10, 8), (6, 4)])
def test_realigned_source_ends_at_allocation_end(nbx, oracle, torch_gpu, dtype, nsrc):
    """every source is its own hipMalloc of exactly 1 MiB (a page
    multiple) and its range ends exactly at the allocation's end, at an offset
    that differs from the destination's — so the realigning kernel's last
    packs (the lane-0 extra pack, the clamped indices) sit right at the edge.
    The result must equal the oracle (and the kernel must not fault: every
    16-B pack it loads holds a byte of the source range)."""
    torch = torch_gpu
    hip = _hip()
    eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
    size = 1 << 20
    bufs = []
    try:
        srcs, ptrs = [], []
        for k in range(nsrc):
            p = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(p), size) == 0
            bufs.append(p.value)
            off = (4 + 3 * k * eb) % 16 or eb            # source start mod 16, never 0 here
            count = (size - 4096 - off) // eb            # range ends at the allocation end
            srcs.append(None)
            ptrs.append((p.value, off, count))
        count = min(c for _, _, c in ptrs)
        host = oracle.random_inputs(dtype, nsrc, count, seed=4000 + dtype * 10 + nsrc)
        sp = []
        for (b, _, _), h in zip(ptrs, host):
            start = b + size - count * eb                # last byte of the range = last byte of the allocation
            assert hip.hipMemcpy(ctypes.c_void_p(start), h.ctypes.data, count * eb, 1) == 0   # H2D
            sp.append(start)
        out = torch.full((count * eb + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        dp = out.data_ptr() + (0 if (sp[0] % 16) else eb)    # destination alignment differs from source 0's
        op = nbx.DevRedOpFull()
        nbx.reduce_multi([dp], sp, count, dtype, op, 0, False, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        exp = oracle.reduce_multi(host, dtype, 0, threads=8)[0]
        o = dp - out.data_ptr()
        assert_same(out[o:o + count * eb].cpu().numpy().view(exp.dtype), exp, dtype)
    finally:
        for b in bufs:
            hip.hipFree(ctypes.c_void_p(b))


@pytest.mark.parametrize("dtype", [7, 6, 4])
def test_realigned_sources_runtime_count_kernel(nbx, oracle, torch_gpu, dtype):
    """Launch variant 1 sends misaligned sources to the run-time-source-count
    realigning kernel (kReduceShifted, the fallback of the per-count kernels):
    1-8 sources, every op, several destinations."""
    eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
    offs = list(range(0, 16, eb))
    rng = np.random.default_rng(dtype + 99)
    try:
        nbx.set_launch_config(0, 1)
        for nsrc in range(1, 9):
            for devop in devops_for(dtype):
                count = int(rng.integers(1, 40000))
                srcs = oracle.random_inputs(dtype, nsrc, count, seed=nsrc * 31 + devop)
                src_off = [offs[(k * 3 + devop + 1) % len(offs)] for k in range(nsrc)]
                ndst = 1 + (nsrc + devop) % 3
                arg = op_arg(oracle, dtype, devop, rng)
                run_case(nbx, oracle, torch_gpu, srcs, dtype, devop, arg, npre=min(2, nsrc) if devop == 3 else 0,
                         post=devop == 4, ndst=ndst, src_off=src_off, dst_off=[offs[devop % len(offs)]] * ndst)
    finally:
        nbx.set_launch_config(0, 0)


@pytest.mark.parametrize("dtype", [2, 7, 9])
def test_two_destinations(nbx, oracle, torch_gpu, dtype):
    srcs = oracle.random_inputs(dtype, 4, 70001, seed=21)
    run_case(nbx, oracle, torch_gpu, srcs, dtype, 0, 0, ndst=2)


@pytest.mark.parametrize("dtype,ndst,nsrc", [(7, 8, 8), (7, 3, 2), (6, 5, 8), (2, 8, 3), (4, 7, 4), (10, 4, 8)])
def test_many_destinations(nbx, oracle, torch_gpu, dtype, ndst, nsrc):
    """Up to NBX_MAX_DSTS = 8 destinations (the direct schedules' push-gather:
    local output + 7 peers), mixed shared misalignment included."""
    srcs = oracle.random_inputs(dtype, nsrc, 50021, seed=ndst * 10 + nsrc)
    run_case(nbx, oracle, torch_gpu, srcs, dtype, 0, 0, ndst=ndst)
    eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
    off = (3 * eb) % 16
    run_case(nbx, oracle, torch_gpu, srcs, dtype, 0, 0, ndst=ndst, src_off=[off] * nsrc, dst_off=[off] * ndst)
    run_case(nbx, oracle, torch_gpu, srcs, dtype, 0, 0, ndst=ndst, src_off=[off] * nsrc,
             dst_off=[(off + eb * d) % 16 for d in range(ndst)])   # mixed alignments: element kernel


@pytest.mark.parametrize("nsrc", [9, 15, 16, 20, 32, 64])
def test_many_sources_multipass(nbx, oracle, torch_gpu, nsrc):
    srcs = oracle.random_inputs(7, nsrc, 30011, seed=nsrc)
    run_case(nbx, oracle, torch_gpu, srcs, 7, 0, 0)
    scal = int(np.float32(1.0 / nsrc).view(np.uint32))
    run_case(nbx, oracle, torch_gpu, srcs, 7, 3, scal, npre=nsrc - 3, ndst=2)
    isrcs = oracle.random_inputs(2, nsrc, 30011, seed=nsrc)
    run_case(nbx, oracle, torch_gpu, isrcs, 2, 4, nsrc, post=True)


@pytest.mark.parametrize("dtype", [0, 6, 7, 8, 9, 10])
def test_device_resident_scalar(nbx, oracle, torch_gpu, dtype):
    """ncclScalarDevice: the kernel dereferences the PreMulSum scalar (common.h:100-119)."""
    arg = oracle.host_to_dev_redop(4, dtype, 5)[1] if dtype in FLOAT_TYPES else 7
    srcs = oracle.random_inputs(dtype, 2, 9999, seed=dtype)
    run_case(nbx, oracle, torch_gpu, srcs, dtype, 3, arg, npre=2, arg_on_device=True)


def test_in_place(nbx, oracle, torch_gpu):
    """dst == srcs[0] (in-place all-reduce shape)."""
    torch = torch_gpu
    srcs = oracle.random_inputs(7, 4, 100003, seed=1)
    exp = oracle.reduce_multi(srcs, 7, 0)[0]
    ts = [torch.from_numpy(s.copy()).cuda() for s in srcs]
    op = nbx.DevRedOpFull()
    nbx.reduce_multi([ts[0].data_ptr()], [t.data_ptr() for t in ts], srcs[0].size, 7, op, 0, False,
                     torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert_same(ts[0].cpu().numpy(), exp, 7)


def run_batch(nbx, oracle, torch, dtype, devop, arg, buckets, npre=0, post=False):
    """nbxReduceMultiBatch over buckets [(nsrc, ndst, count, src_off, dst_off, seed)], each
    checked bit-exact against the oracle's single-bucket fold, guard bytes untouched."""
    dev = Dev(torch)
    st = oracle.NP_STORAGE[dtype]
    eb = np.dtype(st).itemsize
    calls, cases = [], []
    for nsrc, ndst, count, so, do, seed in buckets:
        srcs = oracle.random_inputs(dtype, nsrc, count, seed=seed)
        sp = [dev.upload(x, so) for x in srcs]
        outs = [dev.alloc(count * eb, do) for _ in range(ndst)]
        calls.append(([p for _, p in outs], sp, count))
        cases.append((srcs, outs, do, count))
    op = nbx.DevRedOpFull()
    op.op = devop
    op.scalarArg = arg
    nbx.reduce_multi_batch(calls, dtype, op, npre, post, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for srcs, outs, do, count in cases:
        exp = oracle.reduce_multi(srcs, dtype, devop, arg, npre, post, n_dsts=1, threads=8)[0]
        for t, _ in outs:
            assert_same(Dev.download(t, do, count * eb, st), exp, dtype)
            assert (t[do + count * eb:].cpu().numpy() == 0xA5).all() and (t[:do].cpu().numpy() == 0xA5).all()


@pytest.mark.parametrize("form", [0, 2])
@pytest.mark.parametrize("dtype", ALL_TYPES)
def test_batch_all_types_ops(nbx, oracle, torch_gpu, dtype, form):
    """Batched buckets: every op, ragged sizes (below one pack, one tile +- 1,
    several tiles), 1-8 sources and 1-3 destinations in one call — through the
    kernel-argument tables (form 0) and the work-list kernel (form 2)."""
    lib = nbx.load_library()
    prev = lib.nbxDebugSetBatchMode(form)
    try:
        rng = np.random.default_rng(dtype)
        eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
        epp = 16 // eb
        for devop in devops_for(dtype):
            arg = op_arg(oracle, dtype, devop, rng)
            buckets = []
            for i, count in enumerate([1, epp - 1, epp, 256 * epp - 1, 256 * epp + 1, 3001, 70001]):
                nsrc = 1 + (i + devop) % 8
                buckets.append((nsrc, 1 + i % 3, count, 0, 0, 100 * dtype + 10 * devop + i))
            run_batch(nbx, oracle, torch_gpu, dtype, devop, arg, buckets, npre=2 if devop == 3 else 0,
                      post=devop == 4)
    finally:
        lib.nbxDebugSetBatchMode(prev)


@pytest.mark.parametrize("dtype", [6, 9, 7, 4])
def test_batch_many_buckets_and_alignments(nbx, oracle, torch_gpu, dtype):
    """More buckets than one launch holds (> 16 per source count), shared
    misalignments (head elements), mixed alignments and > 8 sources (the
    single-bucket fallbacks) in one call."""
    eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
    rng = np.random.default_rng(7)
    buckets = []
    for i in range(40):
        nsrc = 8 if i < 20 else int(rng.integers(1, 9))
        off = int(rng.integers(0, 16 // eb)) * eb
        buckets.append((nsrc, 1 + i % 2, int(rng.integers(1, 40000)), off, off, 1000 + i))
    buckets.append((3, 1, 5000, 0, eb % 16 if eb < 16 else 0, 77))   # mixed alignment
    buckets.append((12, 2, 9000, 0, 0, 78))                           # multi-pass
    run_batch(nbx, oracle, torch_gpu, dtype, 0, 0, buckets)


def test_batch_table_overflow(nbx, oracle, torch_gpu):
    """More buckets than one kernel-argument table holds (101 two-source or 28
    eight-source/eight-destination records): the table is launched when full
    and packing resumes."""
    rng = np.random.default_rng(11)
    buckets = [(2, 1, int(rng.integers(1, 3000)), 0, 0, 2000 + i) for i in range(150)]
    buckets += [(8, 8, int(rng.integers(1, 3000)), 4, 4, 3000 + i) for i in range(35)]
    run_batch(nbx, oracle, torch_gpu, 7, 0, 0, buckets)
    run_batch(nbx, oracle, torch_gpu, 2, 4, 3, buckets[140:160], post=True)


@pytest.mark.parametrize("dtype,nsrc", [(7, 8), (6, 4), (9, 5), (4, 6)])
def test_batch_large_sets(nbx, oracle, torch_gpu, dtype, nsrc):
    """Large batches of 4-8 sources (more packs in total than one big tile per
    CU): ragged bucket sizes, shared misalignments, several destinations."""
    eb = np.dtype(oracle.NP_STORAGE[dtype]).itemsize
    rng = np.random.default_rng(nsrc)
    buckets = []
    for i in range(24):
        count = int(rng.integers(200000, 600000)) // eb   # bytes per input -> elements
        off = int(rng.integers(0, 16 // eb)) * eb
        buckets.append((nsrc, 1 + i % 3, count, off, off, 500 + i))
    run_batch(nbx, oracle, torch_gpu, dtype, 0, 0, buckets)


@pytest.mark.parametrize("form", [1, 2])
@pytest.mark.parametrize("dtype", [7, 6, 9])
def test_batch_device_scalar_and_graph_replay(nbx, oracle, torch_gpu, dtype, form):
    """Batched PreMulSum with the scalar in device memory (dereferenced by the
    batch kernel while it runs), captured into a HIP graph and replayed after
    the scalar and the inputs change: the kernel-argument table is captured by
    value (form 1: four buckets use it), the work-list table (form 2) is owned
    by the graph; the scalar and data are read at replay time."""
    lib = nbx.load_library()
    prev = lib.nbxDebugSetBatchMode(form)
    try:
        _batch_scalar_graph(nbx, oracle, torch_gpu, dtype)
    finally:
        lib.nbxDebugSetBatchMode(prev)


def _batch_scalar_graph(nbx, oracle, torch, dtype):
    st_np = oracle.NP_STORAGE[dtype]
    eb = np.dtype(st_np).itemsize
    counts = [5000, 40000, 123, 77777]
    nsrc = 3
    dev = Dev(torch)
    srcs = [[torch.empty(c * eb, dtype=torch.uint8, device="cuda") for _ in range(nsrc)] for c in counts]
    outs = [torch.empty(c * eb, dtype=torch.uint8, device="cuda") for c in counts]
    scal = torch.zeros(8, dtype=torch.uint8, device="cuda")
    op = nbx.DevRedOpFull()
    op.op, op.scalarArgIsPtr, op.scalarArg = 3, 1, scal.data_ptr()
    buckets = [([o.data_ptr()], [t.data_ptr() for t in ss], c) for ss, o, c in zip(srcs, outs, counts)]
    s = torch.cuda.Stream()

    def fill(it):
        host = []
        for k, (ss, c) in enumerate(zip(srcs, counts)):
            xs = oracle.random_inputs(dtype, nsrc, c, seed=100 * it + k)
            for t, x in zip(ss, xs):
                t.copy_(torch.from_numpy(x.view(np.uint8).copy()))
            host.append(xs)
        arg = oracle.host_to_dev_redop(4, dtype, 2 + it)[1]   # Avg scalar 1/(2+it)
        scal.copy_(torch.from_numpy(np.array([arg], dtype=np.uint64).view(np.uint8)))
        return host, arg

    host, arg = fill(0)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        nbx.reduce_multi_batch(buckets, dtype, op, 1, False, s.cuda_stream)   # eager
    s.synchronize()
    for xs, o in zip(host, outs):
        exp = oracle.reduce_multi(xs, dtype, 3, arg, 1, False)[0]
        assert_same(o.cpu().numpy().view(st_np), exp, dtype)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        nbx.reduce_multi_batch(buckets, dtype, op, 1, False, s.cuda_stream)
    for it in (1, 2):
        host, arg = fill(it)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        for xs, o in zip(host, outs):
            exp = oracle.reduce_multi(xs, dtype, 3, arg, 1, False)[0]
            assert_same(o.cpu().numpy().view(st_np), exp, dtype)
    del dev


def test_batch_mixed_bucket_sweep_fp16_bf16(nbx, oracle, torch_gpu):
    """Config C shape: 8-source fp16 and bf16 sums over 1..16 MiB buckets in one
    batch — by default the buckets that fill the GPU alone take the big-tile
    single-bucket kernel; launch variant 1 puts every bucket in the batch kernel."""
    try:
        for variant in (0, 1):
            nbx.set_launch_config(0, variant)
            for dtype in (6, 9):
                buckets = [(8, 1, (mib << 20) // 2, 0, 0, mib + variant) for mib in (1, 2, 4, 8, 16)]
                run_batch(nbx, oracle, torch_gpu, dtype, 0, 0, buckets)
    finally:
        nbx.set_launch_config(0, 0)


@pytest.mark.parametrize("mode", [1, 0])
def test_batch_work_list_and_kernarg_forms(nbx, oracle, torch_gpu, mode):
    """Both launch forms of nbxReduceMultiBatch on the same ragged sets: work
    lists (mode 1: records in a pinned host table, ~370 buckets per table, so
    450 two-source buckets need two launches) and kernel-argument tables (mode
    0: 101 two-source / 28 eight-source-eight-destination records per launch)."""
    lib = nbx.load_library()
    prev = lib.nbxDebugSetBatchMode(mode)
    try:
        rng = np.random.default_rng(31 + mode)
        buckets = [(2, 1, int(rng.integers(1, 5000)), 0, 0, 4000 + i) for i in range(450)]
        buckets += [(8, 8, int(rng.integers(1, 20000)), 8, 8, 5000 + i) for i in range(40)]
        buckets += [(5, 2, int(rng.integers(1, 300000)), 4, 4, 6000 + i) for i in range(6)]
        run_batch(nbx, oracle, torch_gpu, 7, 0, 0, buckets)
        run_batch(nbx, oracle, torch_gpu, 6, 0, 0, [(8, 1, 32768, 0, 0, 7000 + i) for i in range(128)])
    finally:
        lib.nbxDebugSetBatchMode(prev)


def test_batch_work_list_slots_and_graph_ownership(nbx, oracle, torch_gpu):
    """Work-list table slots: eager calls recycle them (with more calls in
    flight than the arena's 128 slots the rest fall back to kernel-argument
    batches, never wait), a call captured into a graph keeps its slot for the
    graph's lifetime — eager calls issued between replays never overwrite it —
    and every replay reads it in place."""
    torch = torch_gpu
    lib = nbx.load_library()
    dev_id = torch.cuda.current_device()
    prev = lib.nbxDebugSetBatchMode(1)
    try:
        dtype, nsrc = 7, 4
        counts = [3000, 70000, 5, 40001] * 5   # 20 buckets: more than the kernel-argument form takes (16)
        srcs = [[torch.empty(c, dtype=torch.float32, device="cuda") for _ in range(nsrc)] for c in counts]
        outs = [torch.empty(c, dtype=torch.float32, device="cuda") for c in counts]
        buckets = [([o.data_ptr()], [t.data_ptr() for t in ss], c) for ss, o, c in zip(srcs, outs, counts)]
        other_in = [torch.rand(1000, device="cuda") for _ in range(2)]
        other_out = [torch.empty(1000, device="cuda") for _ in range(20)]
        other = [([o.data_ptr()], [t.data_ptr() for t in other_in], 1000) for o in other_out]
        op = nbx.DevRedOpFull()
        s = torch.cuda.Stream()

        def fill(it):
            host = []
            for k, (ss, c) in enumerate(zip(srcs, counts)):
                xs = oracle.random_inputs(dtype, nsrc, c, seed=300 * it + k)
                for t, x in zip(ss, xs):
                    t.copy_(torch.from_numpy(x))
                host.append(xs)
            return host

        def check(host):
            for xs, o in zip(host, outs):
                assert_same(o.cpu().numpy(), oracle.reduce_multi(xs, dtype, 0)[0], dtype)

        host = fill(0)
        torch.cuda.synchronize()
        fb0 = lib.nbxDebugBatchListSlots(dev_id, 3)
        # hold the stream until every call below is enqueued, so more than 128
        # slots are in flight however fast or slow the host is
        hold = lib.nbxDebugHoldStream(ctypes.c_void_p(s.cuda_stream), 60_000)
        assert hold >= 0
        try:
            with torch.cuda.stream(s):
                for _ in range(300):   # > 128 slots in flight: the rest fall back to kernel-argument tables
                    nbx.reduce_multi_batch(buckets, dtype, op, 0, False, s.cuda_stream)
        finally:
            assert lib.nbxDebugReleaseStream(hold) == 0
        s.synchronize()
        check(host)
        assert lib.nbxDebugBatchListSlots(dev_id, 3) > fb0   # the fallback ran, and came out right
        with torch.cuda.stream(s):
            for _ in range(20):   # each eager call returns a few completed slots to the free pool
                nbx.reduce_multi_batch(buckets, dtype, op, 0, False, s.cuda_stream)
                s.synchronize()
        assert lib.nbxDebugBatchListSlots(dev_id, 0) > 0
        owned0 = lib.nbxDebugBatchListSlots(dev_id, 2)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            nbx.reduce_multi_batch(buckets, dtype, op, 0, False, s.cuda_stream)
        assert lib.nbxDebugBatchListSlots(dev_id, 2) == owned0 + 1
        for it in (1, 2):
            host = fill(it)
            with torch.cuda.stream(s):
                for _ in range(100):   # recycles every other slot, never the graph's
                    nbx.reduce_multi_batch(other, dtype, op, 0, False, s.cuda_stream)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            check(host)
        del g
        torch.cuda.synchronize()
        # the graph's slot comes back once the graph is destroyed (if the
        # runtime runs user-object destructors; otherwise it stays owned)
        assert lib.nbxDebugBatchListSlots(dev_id, 2) in (owned0, owned0 + 1)
    finally:
        lib.nbxDebugSetBatchMode(prev)


def test_invalid_arguments(nbx, torch_gpu):
    torch = torch_gpu
    a = torch.zeros(64, device="cuda")
    p = a.data_ptr()
    op = nbx.DevRedOpFull()
    E = nbx.ncclResult.ncclInvalidArgument
    assert nbx.reduce_multi_raw([p], [], 16, 7, op) == E                       # no sources
    assert nbx.reduce_multi_raw([p], [p] * 65, 16, 7, op) == E                 # > NBX_MAX_SRCS (64)
    assert nbx.reduce_multi_raw([p] * 9, [p], 16, 7, op) == E                  # > NBX_MAX_DSTS (8)
    assert nbx.reduce_multi_raw([p], [p], 16, 12, op) == E                     # bad datatype
    op.op = 4
    op.scalarArg = 2
    assert nbx.reduce_multi_raw([p], [p], 16, 7, op) == E                      # SumPostDiv on float
    op.op = 0
    assert nbx.reduce_multi_raw([p], [p + 2], 16, 7, op) == E                  # not element-aligned
    assert nbx.reduce_multi_raw([0], [p], 16, 7, op) == E                      # NULL dst


@pytest.mark.parametrize("nsrc,alias", [(9, 8), (9, 0), (16, 15), (20, 9), (20, 19), (64, 63)])
def test_multipass_destination_aliases_a_source(nbx, oracle, torch_gpu, nsrc, alias):
    """More than 8 sources fold in passes; when the destination IS a source a
    later pass reads (in-place collectives past 8 ranks: the rank's own block
    is last in fold order), the partial goes through scratch memory and the
    result is still the oracle's left fold (this used to be
    ncclInvalidArgument)."""
    torch = torch_gpu
    count = 100003
    srcs = oracle.random_inputs(7, nsrc, count, seed=300 + nsrc + alias)
    ts = [torch.from_numpy(x.copy()).cuda() for x in srcs]
    op = nbx.DevRedOpFull()
    nbx.reduce_multi([ts[alias].data_ptr(), ], [t.data_ptr() for t in ts], count, 7, op, 0, False,
                     torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    exp = oracle.reduce_multi(srcs, 7, 0, threads=8)[0]
    assert_same(ts[alias].cpu().numpy(), exp, 7)


def test_config_b_full_size_bit_exact(nbx, oracle, torch_gpu):
    """BASELINE config B at full size: 8 x 256 MiB fp32 sum, bit-exact vs the
    multithreaded oracle on the same seeded buffers."""
    torch = torch_gpu
    n = 64 << 20
    g = torch.Generator(device="cuda").manual_seed(1234)
    ts = [torch.rand(n, device="cuda", generator=g) * 2 - 1 for _ in range(8)]
    out = torch.empty(n, device="cuda")
    op = nbx.DevRedOpFull()
    nbx.reduce_multi([out.data_ptr()], [t.data_ptr() for t in ts], n, 7, op, 0, False,
                     torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    host = [t.cpu().numpy() for t in ts]
    exp = oracle.reduce_multi(host, 7, 0, threads=16)[0]
    got = out.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))


def test_config_e_int64_max_and_fp8_sum(nbx, oracle, torch_gpu):
    """BASELINE config E shapes on one GPU: int64 ncclMax over 16,777,216
    elements (128 MiB) and fp8 e4m3 ncclSum over 134,217,728 elements
    (128 MiB), 8 sources each, bit-exact vs the oracle (fp8: this build's
    definition, parity unpinned vs the reference)."""
    torch = torch_gpu
    stream = torch.cuda.current_stream().cuda_stream
    for dtype, n, opcode in ((4, 16 << 20, 2), (10, 128 << 20, 0)):
        srcs = oracle.random_inputs(dtype, 8, n, seed=77) if dtype == 4 else \
            [np.random.default_rng(77 + s).integers(0, 256, n, dtype=np.uint8) for s in range(8)]
        if dtype == 10:
            for s in srcs:
                s[(s & 0x7F) == 0x7F] &= 0xF7   # finite codes
        devop, arg = oracle.host_to_dev_redop(opcode, dtype, 8)
        ts = [torch.from_numpy(s.view(np.uint8)).cuda() for s in srcs]
        out = torch.empty_like(ts[0])
        op = nbx.DevRedOpFull()
        op.op, op.scalarArg = devop, arg
        nbx.reduce_multi([out.data_ptr()], [t.data_ptr() for t in ts], n, dtype, op, 0, False, stream)
        torch.cuda.synchronize()
        exp = oracle.reduce_multi(srcs, dtype, devop, arg, threads=16)[0]
        assert_same(out.cpu().numpy().view(exp.dtype), exp, dtype)


def test_fp8_exhaustive_pairs(nbx, oracle, torch_gpu):
    """Every (a, b) pair of fp8 codes through sum / prod / min / max / premulsum,
    both formats: pins the device fp8 narrowing against the oracle codec."""
    a = np.repeat(np.arange(256, dtype=np.uint8), 256)
    b = np.tile(np.arange(256, dtype=np.uint8), 256)
    for dtype in (10, 11):
        for devop, arg in ((0, 0), (1, 0), (2, 0), (2, 0xFF), (3, oracle.host_to_dev_redop(4, dtype, 3)[1])):
            run_case(nbx, oracle, torch_gpu, [a, b], dtype, devop, arg, npre=1 if devop == 3 else 0)


def test_half_bf16_exhaustive_against_one(nbx, oracle, torch_gpu):
    """All 65536 f16 / bf16 codes against a spread of second operands."""
    a = np.arange(65536, dtype=np.uint16)
    for dtype in (6, 9):
        for seed in range(3):
            b = np.random.default_rng(seed).integers(0, 65536, 65536, dtype=np.uint16)
            for devop, arg in ((0, 0), (1, 0), (2, 0), (2, 0xFFFF)):
                run_case(nbx, oracle, torch_gpu, [a, b], dtype, devop, arg)


@pytest.mark.parametrize("dtype,devop", [(7, 0), (6, 0), (9, 3), (2, 4), (10, 0), (8, 2)])
@pytest.mark.parametrize("count", [1, 1000, (1 << 20) + 13, 5 << 20])
def test_host_staged_reduce(nbx, oracle, torch_gpu, monkeypatch, dtype, devop, count):
    """nbxReduceMultiHost: pageable numpy buffers in and out, chunked through the
    device ring (small chunk size forces many chunks and slot reuse)."""
    monkeypatch.setenv("NBX_HOST_CHUNK_BYTES", str(256 << 10))
    rng = np.random.default_rng(count + dtype)
    nsrc = 3
    srcs = oracle.random_inputs(dtype, nsrc, count, seed=int(rng.integers(1 << 20)))
    arg = op_arg(oracle, dtype, devop, rng)
    npre = 2 if devop == 3 else 0
    st = oracle.NP_STORAGE[dtype]
    outs = [np.full(count, 0x5A, dtype=np.uint8 if np.dtype(st).itemsize == 1 else st) for _ in range(2)]
    outs = [o.view(st) for o in outs]
    op = nbx.DevRedOpFull()
    op.op, op.scalarArg = devop, arg
    nbx.reduce_multi_host([o.ctypes.data for o in outs], [s.ctypes.data for s in srcs], count, dtype, op, npre,
                          devop == 4, torch_gpu.cuda.current_stream().cuda_stream)
    exp = oracle.reduce_multi(srcs, dtype, devop, arg, npre, devop == 4, threads=8)[0]
    for o in outs:
        assert_same(o, exp, dtype)


@pytest.mark.parametrize("mode", ["auto", "zerocopy", "staged"])
@pytest.mark.parametrize("dtype,devop,count", [(7, 0, (1 << 20) + 13), (6, 3, 5000), (4, 2, 3 << 20), (2, 4, 777)])
def test_host_pinned_zero_copy(nbx, oracle, torch_gpu, monkeypatch, mode, dtype, devop, count):
    """nbxReduceMultiHost on pinned (torch pin_memory) buffers: zero-copy — the
    kernel reads and writes host memory over PCIe — under auto / zerocopy, the
    staging ring under staged; a shared misalignment included (offset views)."""
    torch = torch_gpu
    monkeypatch.setenv("NBX_HOST_MODE", mode)
    monkeypatch.setenv("NBX_HOST_CHUNK_BYTES", str(256 << 10))
    rng = np.random.default_rng(count + dtype)
    nsrc = 4
    srcs = oracle.random_inputs(dtype, nsrc, count, seed=int(rng.integers(1 << 20)))
    arg = op_arg(oracle, dtype, devop, rng)
    npre = 2 if devop == 3 else 0
    st = oracle.NP_STORAGE[dtype]
    eb = np.dtype(st).itemsize
    off = eb if eb < 16 else 0   # every pointer one element past 16-B alignment
    pins = [torch.empty(count * eb + 64, dtype=torch.uint8).pin_memory() for _ in range(nsrc + 2)]
    for p, x in zip(pins, srcs):
        p.numpy()[off:off + count * eb] = x.view(np.uint8)
    for p in pins[nsrc:]:
        p.numpy()[:] = 0x5A
    op = nbx.DevRedOpFull()
    op.op, op.scalarArg = devop, arg
    sp = [p.data_ptr() + off for p in pins[:nsrc]]
    dp = [p.data_ptr() + off for p in pins[nsrc:]]
    nbx.reduce_multi_host(dp, sp, count, dtype, op, npre, devop == 4, torch.cuda.current_stream().cuda_stream)
    exp = oracle.reduce_multi(srcs, dtype, devop, arg, npre, devop == 4, threads=8)[0]
    for p in pins[nsrc:]:
        got = p.numpy()[off:off + count * eb].view(st)
        assert_same(got, exp, dtype)
        assert (p.numpy()[:off] == 0x5A).all() and (p.numpy()[off + count * eb:] == 0x5A).all()


def test_host_zero_copy_refuses_pageable(nbx, torch_gpu, monkeypatch):
    """NBX_HOST_MODE=zerocopy with a pageable buffer: ncclInvalidArgument, nothing run."""
    monkeypatch.setenv("NBX_HOST_MODE", "zerocopy")
    a = np.ones(1024, dtype=np.float32)
    o = np.zeros(1024, dtype=np.float32)
    with pytest.raises(nbx.NcclError):
        nbx.reduce_multi_host([o.ctypes.data], [a.ctypes.data], 1024, 7, nbx.DevRedOpFull(), 0, False,
                              torch_gpu.cuda.current_stream().cuda_stream)
    assert (o == 0).all()


def test_beyond_32bit_counts(nbx, torch_gpu):
    """Maximum sizes: element counts and byte offsets past 2^32 (u8 sum of
    4 GiB + 37 elements; f32 sum of 2^30 + 5 elements = 4 GiB + 20 B per
    buffer), plus a 1-element head from a shared misalignment, checked in full
    against torch on the GPU (u8 + wraps like the SWAR functor; one f32 add is
    correctly rounded either way)."""
    torch = torch_gpu
    st = torch.cuda.current_stream().cuda_stream
    n = (1 << 32) + 37
    g = torch.Generator(device="cuda").manual_seed(99)
    a = torch.randint(0, 256, (n + 1,), dtype=torch.uint8, device="cuda", generator=g)
    b = torch.randint(0, 256, (n + 1,), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty(n + 1, dtype=torch.uint8, device="cuda")
    op = nbx.host_to_dev_redop(nbx.ncclRedOp.ncclSum, nbx.ncclDataType.ncclUint8, 1)
    # one byte in: every pointer shares misalignment 1 (head element + aligned body + tail)
    nbx.reduce_multi([out.data_ptr() + 1], [a.data_ptr() + 1, b.data_ptr() + 1], n, 1, op, 0, False, st)
    torch.cuda.synchronize()
    assert torch.equal(out[1:], a[1:] + b[1:])
    del a, b, out
    torch.cuda.empty_cache()
    m = (1 << 30) + 5
    x = torch.rand(m, device="cuda", generator=g)
    y = torch.rand(m, device="cuda", generator=g)
    o = torch.empty_like(x)
    op = nbx.host_to_dev_redop(nbx.ncclRedOp.ncclSum, nbx.ncclDataType.ncclFloat32, 1)
    nbx.reduce_multi([o.data_ptr()], [x.data_ptr(), y.data_ptr()], m, 7, op, 0, False, st)
    torch.cuda.synchronize()
    assert torch.equal(o, x + y)


@pytest.fixture
def dynamic_tiles_always(nbx):
    """Every big-tile launch takes the dynamic schedule (by default only
    launches of >= 16 tiles per workgroup do, nbxDebugSetDynMinTiles), so the
    tests below exercise the counters at sizes the oracle checks quickly."""
    lib = nbx.load_library()
    lib.nbxDebugSetDynMinTiles.restype = ctypes.c_int
    prev = lib.nbxDebugSetDynMinTiles(1)
    assert prev >= 1
    yield
    lib.nbxDebugSetDynMinTiles(prev)


def test_dynamic_tiles_across_streams_and_graphs(nbx, oracle, torch_gpu, dynamic_tiles_always):
    """Big-tile launches take their tiles from a per-stream counter whose
    per-launch base the host tracks (nbx_tiles.h): many launches of different
    sizes on three streams at once, a > 8-source multi-pass call, and a graph
    capture (static tiles) replayed between eager calls on the same stream all
    stay bit-exact."""
    torch = torch_gpu
    dtype = 7
    streams = [torch.cuda.Stream() for _ in range(3)]
    sizes = [(1 << 20) + 17, 3 << 20, (1 << 21) + 4099]
    cases = []
    for k, n in enumerate(sizes):
        srcs = oracle.random_inputs(dtype, 8, n, seed=900 + k)
        exp = oracle.reduce_multi(srcs, dtype, 0, threads=8)[0]
        ts = [torch.from_numpy(x).cuda() for x in srcs]
        out = torch.empty(n, dtype=torch.float32, device="cuda")
        cases.append((ts, out, exp, n))
    op = nbx.DevRedOpFull()
    torch.cuda.synchronize()
    for rep in range(12):   # interleaved sizes on three streams, no host sync in between
        for k, (ts, out, exp, n) in enumerate(cases):
            s = streams[(k + rep) % 3]
            with torch.cuda.stream(s):
                out.zero_()
                nbx.reduce_multi([out.data_ptr()], [t.data_ptr() for t in ts], n, dtype, op, 0, False, s.cuda_stream)
            for s2 in streams:   # the next writer of `out` waits for this one
                s2.wait_stream(s)
    torch.cuda.synchronize()
    for ts, out, exp, n in cases:
        assert_same(out.cpu().numpy(), exp, dtype)
    # multi-pass (> 8 sources) and a captured launch replayed between eager ones
    srcs = oracle.random_inputs(dtype, 12, (1 << 21) + 5, seed=950)
    exp = oracle.reduce_multi(srcs, dtype, 0, threads=8)[0]
    ts = [torch.from_numpy(x).cuda() for x in srcs]
    out = torch.empty(exp.size, dtype=torch.float32, device="cuda")
    s = streams[0]
    call = lambda: nbx.reduce_multi([out.data_ptr()], [t.data_ptr() for t in ts], exp.size, dtype, op, 0, False,
                                    s.cuda_stream)
    with torch.cuda.stream(s):
        call()
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        call()
    for _ in range(3):
        with torch.cuda.stream(s):
            out.zero_()
            g.replay()
            call()
            g.replay()
        s.synchronize()
        assert_same(out.cpu().numpy(), exp, dtype)


def test_dynamic_tiles_threads_sharing_a_stream(nbx, oracle, torch_gpu, dynamic_tiles_always):
    """Host threads racing nbxReduceMulti calls onto ONE stream: each call
    reads its stream counter's base and launches under one lock, so bases stay
    in enqueue order and every call's tiles are its own (ctypes drops the GIL
    during the call, so the threads really overlap)."""
    import threading
    torch = torch_gpu
    dtype = 7
    s = torch.cuda.Stream()
    n = (1 << 20) + 333
    srcs = oracle.random_inputs(dtype, 8, n, seed=977)
    exp = oracle.reduce_multi(srcs, dtype, 0, threads=8)[0]
    ts = [torch.from_numpy(x).cuda() for x in srcs]
    outs = [torch.zeros(n, dtype=torch.float32, device="cuda") for _ in range(16)]
    torch.cuda.synchronize()
    lib = nbx.load_library()
    sp = (ctypes.c_void_p * 8)(*[t.data_ptr() for t in ts])
    op = nbx.DevRedOpFull()
    errs = []

    def worker(k):
        try:
            for rep in range(6):
                o = outs[(k * 4 + rep) % 16]
                dp = (ctypes.c_void_p * 1)(o.data_ptr())
                rc = lib.nbxReduceMulti(dp, 1, sp, 8, ctypes.c_size_t(n), dtype, op, 0, 0, ctypes.c_void_p(s.cuda_stream))
                if rc != 0:
                    errs.append(rc)
        except Exception as e:   # pragma: no cover - reported below
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    s.synchronize()
    assert not errs, errs
    for o in outs:
        assert_same(o.cpu().numpy(), exp, dtype)


def test_dynamic_counters_with_stream_churn(nbx, oracle, torch_gpu, dynamic_tiles_always):
    """Per-stream counters are keyed by the stream handle, and HIP hands a
    destroyed stream's handle to the next stream created. That is safe because
    hipStreamDestroy returns only after the stream's work completed
    (scripts/probe_stream_destroy.py): streams are created, given dynamic
    launches (big-tile tile counters and the realigning kernel's class
    counters) and destroyed with that work still queued, one after another;
    every output stays bit-exact and the counters in use stay few."""
    torch = torch_gpu
    lib = nbx.load_library()
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    lib.nbxDebugDynStreamSlots.argtypes = [ctypes.c_int, ctypes.c_int]
    dtype = 7
    n = (1 << 20) + 37
    srcs = oracle.random_inputs(dtype, 8, n + 1, seed=991)
    exp_big = oracle.reduce_multi([x[:n] for x in srcs], dtype, 0, threads=8)[0]
    exp_shift = oracle.reduce_multi([x[1:n + 1] if i % 2 else x[:n] for i, x in enumerate(srcs[:4])], dtype, 0,
                                    threads=8)[0]
    ts = [torch.from_numpy(x).cuda() for x in srcs]
    big_src = [t.data_ptr() for t in ts]
    shift_src = [t.data_ptr() + (4 if i % 2 else 0) for i, t in enumerate(ts[:4])]   # mixed alignment
    iters = 16
    outs = [(torch.zeros(n, dtype=torch.float32, device="cuda"), torch.zeros(n, dtype=torch.float32, device="cuda"))
            for _ in range(iters)]
    op = nbx.DevRedOpFull()
    dev = torch.cuda.current_device()
    torch.cuda.synchronize()
    used0 = [lib.nbxDebugDynStreamSlots(dev, w) for w in (0, 1)]
    for k in range(iters):
        st = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) == 0
        ob, osh = outs[k]
        for _ in range(2):
            nbx.reduce_multi([ob.data_ptr()], big_src, n, dtype, op, 0, False, st.value)
            nbx.reduce_multi([osh.data_ptr()], shift_src, n, dtype, op, 0, False, st.value)
        assert hip.hipStreamDestroy(st) == 0   # with its launches still queued
    torch.cuda.synchronize()
    for ob, osh in outs:
        assert_same(ob.cpu().numpy(), exp_big, dtype)
        assert_same(osh.cpu().numpy(), exp_shift, dtype)
    used1 = [lib.nbxDebugDynStreamSlots(dev, w) for w in (0, 1)]
    assert all(u1 - u0 <= 2 for u0, u1 in zip(used0, used1)), (used0, used1)
