"""C-ABI boundary tests that need no GPU: the library loads, exports every
symbol include/*.h declares (plus the p-prefixed profiling aliases of the NCCL
API, src/include/core.h:17-32), enum values match the reference header, and
the pure host logic (op encoding, argument checks that fail before any device
call, error strings) behaves like the reference."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include")


def declared_functions():
    names = set()
    for h in os.listdir(INCLUDE):
        if not h.endswith(".h"):
            continue
        text = open(os.path.join(INCLUDE, h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s+\*?\s*([A-Za-z_][A-Za-z0-9_]*)\s*\(",
                             text, flags=re.M):
            name = m.group(1)
            if name.startswith(("nccl", "pnccl", "nbx")) and name not in ("ncclResult_t",):
                names.add(name)
    return sorted(names)


def test_headers_declare_expected_api():
    names = declared_functions()
    for must in ("ncclAllReduce", "ncclReduceScatter", "ncclReduce", "ncclCommInitRank", "ncclCommInitAll",
                 "ncclRedOpCreatePreMulSum", "ncclGroupStart", "nbxReduceMulti", "nbxHostToDevRedOp",
                 "pncclAllReduce"):
        assert must in names, must


def test_library_exports_every_declared_symbol(nbx):
    lib = nbx.load_library()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", nbx.library_path()], capture_output=True, text=True,
                         check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert set(declared_functions()) <= exported
    # nothing from the oracle leaks into the product
    assert not any(s.startswith("oracle_") for s in exported)


def test_library_has_gfx950_code_object(nbx):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", nbx.library_path()], capture_output=True,
                         text=True)
    assert ".hip_fatbin" in out.stdout
    blob = open(nbx.library_path(), "rb").read()
    assert b"gfx950" in blob


def test_enum_values_match_reference(nbx):
    # nccl.h.in:37-45, 181-214
    assert [int(v) for v in nbx.ncclResult] == list(range(8))
    assert [int(nbx.ncclRedOp[n]) for n in ("ncclSum", "ncclProd", "ncclMax", "ncclMin", "ncclAvg")] == [0, 1, 2, 3, 4]
    assert int(nbx.ncclDataType.ncclBfloat16) == 9 and int(nbx.ncclDataType.ncclFloat64) == 8
    assert [int(v) for v in nbx.DevRedOp] == [0, 1, 2, 3, 4]   # device.h:26-30


def test_version_and_error_strings(nbx):
    assert nbx.get_version() == 21904
    assert nbx.get_error_string(0) == "no error"
    assert nbx.get_error_string(4).startswith("invalid argument")
    assert nbx.get_error_string(6) == "remote process exited or there was a network error"
    assert nbx.get_error_string(99) == "unknown result code"


@pytest.mark.parametrize("dtype", range(12))
@pytest.mark.parametrize("op", range(5))
@pytest.mark.parametrize("nranks", [1, 3, 8])
def test_host_to_dev_redop_matches_oracle(nbx, oracle, dtype, op, nranks):
    got = nbx.host_to_dev_redop(op, dtype, nranks)
    devop, arg = oracle.host_to_dev_redop(op, dtype, nranks)
    assert (got.op, got.scalarArg, got.scalarArgIsPtr) == (devop, arg, 0)


def test_host_to_dev_redop_rejects_bad_args(nbx):
    lib = nbx.load_library()
    out = nbx.DevRedOpFull()
    assert lib.nbxHostToDevRedOp(ctypes.byref(out), 5, 7, 1) == 4     # user op ids need a comm
    assert lib.nbxHostToDevRedOp(ctypes.byref(out), 0, 12, 1) == 4    # bad type
    assert lib.nbxHostToDevRedOp(None, 0, 7, 1) == 4


def test_reduce_multi_argument_checks_before_device(nbx):
    """Checks that return before any HIP call (same codes on CPU and GPU)."""
    op = nbx.DevRedOpFull()
    E = 4
    fake = 0x10000
    assert nbx.reduce_multi_raw([fake], [], 16, 7, op) == E
    assert nbx.reduce_multi_raw([fake], [fake] * 65, 16, 7, op) == E   # > NBX_MAX_SRCS
    assert nbx.reduce_multi_raw([], [fake], 16, 7, op) == E
    assert nbx.reduce_multi_raw([fake], [fake], 16, -1, op) == E
    op.op = 9
    assert nbx.reduce_multi_raw([fake], [fake], 16, 7, op) == E
    op.op = 4
    op.scalarArg = 4
    assert nbx.reduce_multi_raw([fake], [fake], 16, 7, op) == E      # SumPostDiv float: static_assert in ref
    op.scalarArg = 0
    assert nbx.reduce_multi_raw([fake], [fake], 16, 2, op) == E      # divisor 0
    op.op = 0
    assert nbx.reduce_multi_raw([fake], [fake], 0, 7, op) == 0       # count 0: no-op
    assert nbx.reduce_multi_raw([fake], [fake + 2], 16, 7, op) == E  # not element aligned
    assert nbx.reduce_multi_raw([0], [fake], 16, 7, op) == E         # NULL


def test_reduce_multi_batch_argument_checks_before_device(nbx):
    """nbxReduceMultiBatch checks every bucket before enqueuing anything."""
    op = nbx.DevRedOpFull()
    E = 4
    fake = 0x10000
    good = ([fake + 64], [fake, fake + 128], 16)
    assert nbx.reduce_multi_batch_raw([], 7, op) == 0                          # no buckets: no-op
    assert nbx.reduce_multi_batch_raw([([fake], [fake], 0)] * 3, 7, op) == 0   # empty buckets: no-op
    assert nbx.reduce_multi_batch_raw([good, ([fake], [], 16)], 7, op) == E    # a bucket with no source
    assert nbx.reduce_multi_batch_raw([good, ([], [fake], 16)], 7, op) == E    # ... no destination
    assert nbx.reduce_multi_batch_raw([good, ([fake], [fake] * 65, 16)], 7, op) == E
    assert nbx.reduce_multi_batch_raw([good, ([fake], [fake + 2], 16)], 7, op) == E   # misaligned element
    assert nbx.reduce_multi_batch_raw([good, ([0], [fake], 16)], 7, op) == E   # NULL destination
    assert nbx.reduce_multi_batch_raw([good], -1, op) == E
    op.op = 4
    op.scalarArg = 2
    assert nbx.reduce_multi_batch_raw([good], 7, op) == E                      # SumPostDiv on floats
    lib = nbx.load_library()
    assert lib.nbxReduceMultiBatch(None, 2, 7, nbx.DevRedOpFull(), 0, 0, None) == E
    assert lib.nbxReduceMultiBatch(None, -1, 7, nbx.DevRedOpFull(), 0, 0, None) == E


def test_comm_api_errors_without_device(nbx):
    lib = nbx.load_library()
    uid = nbx.get_unique_id()
    assert uid.internal[:8] == b"NBXUID01"
    h = ctypes.c_void_p()
    assert lib.ncclCommInitRank(ctypes.byref(h), 2, uid, 2) == 4      # rank out of range
    assert lib.ncclCommInitRank(ctypes.byref(h), 0, uid, 0) == 4
    bad = nbx.ncclUniqueId()
    assert lib.ncclCommInitRank(ctypes.byref(h), 1, bad, 0) == 4      # not from ncclGetUniqueId
    assert lib.ncclCommInitRank(ctypes.byref(h), 65, uid, 0) == 4     # > 64 ranks per communicator
    assert lib.ncclAllReduce(None, None, 0, 7, 0, None, None) == 4    # NULL comm (argcheck.cc:28-34)
    assert lib.ncclRedOpDestroy(0, ctypes.c_void_p(1)) == 4           # builtin op
    assert lib.ncclRedOpDestroy(-1, ctypes.c_void_p(1)) == 4          # garbage
    assert lib.ncclCommDestroy(None) == 0
    assert lib.ncclGroupEnd() == 5                                     # not in a group
    assert lib.ncclGroupStart() == 0 and lib.ncclGroupEnd() == 0
    assert lib.ncclGetLastError(None) is not None


def test_p_aliases_are_the_same_functions(nbx):
    lib = nbx.load_library()
    for name in ("ncclAllReduce", "ncclReduceScatter", "ncclGetVersion", "ncclGroupStart"):
        a = ctypes.cast(getattr(lib, name), ctypes.c_void_p).value
        b = ctypes.cast(getattr(lib, "p" + name), ctypes.c_void_p).value
        assert a == b, name


def test_reference_symbols_left_out(nbx):
    """of nccl.h.in's entry points, exactly the non-reducing
    collectives and point-to-point calls are not exported (a binary that
    references them does not resolve against this library)."""
    out = subprocess.run(["nm", "-D", "--defined-only", nbx.library_path()], capture_output=True, text=True,
                         check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines()}
    left_out = {"ncclBcast", "ncclBroadcast", "ncclAllGather", "ncclSend", "ncclRecv"}
    assert not (left_out & exported)
    assert not ({"p" + s for s in left_out} & exported)
    reference_api = {"ncclMemAlloc", "ncclMemFree", "ncclGetVersion", "ncclGetUniqueId", "ncclCommInitRankConfig",
                     "ncclCommInitRank", "ncclCommInitAll", "ncclCommFinalize", "ncclCommDestroy", "ncclCommAbort",
                     "ncclCommSplit", "ncclGetErrorString", "ncclGetLastError", "ncclCommGetAsyncError",
                     "ncclCommCount", "ncclCommCuDevice", "ncclCommUserRank", "ncclRedOpCreatePreMulSum",
                     "ncclRedOpDestroy", "ncclReduce", "ncclAllReduce", "ncclReduceScatter", "ncclGroupStart",
                     "ncclGroupEnd", "ncclCommRegister", "ncclCommDeregister"}   # nccl.h.in:84-434, 31 minus 5
    assert len(reference_api) + len(left_out) == 31
    assert reference_api <= exported and {"p" + s for s in reference_api} <= exported


_UID = []


def _one_rank_uid(nbx):
    """One unique id for every case (a one-rank communicator never connects to its root)."""
    if not _UID:
        _UID.append(nbx.get_unique_id())
    return _UID[0]


@pytest.mark.parametrize("fields,ok", [
    ({"minCTAs": 4}, False),                     # the reference's check: an unset maxCTAs is INT_MIN
    ({"minCTAs": 0, "maxCTAs": 8}, False), ({"maxCTAs": -2}, False), ({"minCTAs": 8, "maxCTAs": 4}, False),
    ({"splitShare": 2}, False), ({"cgaClusterSize": -1}, False), ({"blocking": 3}, False),
    ({"magic": 0x1234}, False),
    ({"maxCTAs": 8}, True), ({"minCTAs": 2, "maxCTAs": 8}, True), ({"splitShare": 1, "cgaClusterSize": 0}, True),
    ({"version": 21600, "minCTAs": 0}, True),    # < 2.17: the CTA fields predate the caller and take defaults
])
def test_config_checks_as_parse_comm_config(nbx, fields, ok):
    """ncclCommInitRankConfig checks the config as parseCommConfig does
    (init.cc:1526-1594) before any device call: bad values are
    ncclInvalidArgument; good ones get past the check (here, with no GPU, the
    call fails later and differently, or succeeds on a GPU box)."""
    lib = nbx.load_library()
    cfg = nbx.ncclConfig.initializer(**fields)
    h = ctypes.c_void_p()
    uid = _one_rank_uid(nbx)
    rc = lib.ncclCommInitRankConfig(ctypes.byref(h), 1, uid, 0, ctypes.byref(cfg))
    inval = int(nbx.ncclResult.ncclInvalidArgument)
    assert (rc != inval) if ok else (rc == inval), rc
    if rc in (0, 7) and h.value:
        lib.ncclCommDestroy(h)
