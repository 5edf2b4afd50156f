"""neuronabox-nccl_amd — Python mirror of the NCCL reduction API over libnbxccl.so.

The product is the C-ABI shared library ``lib/libnbxccl.so`` (HIP kernels for
gfx950 + the NCCL-compatible host layer); this module only binds it with
ctypes so tests, the bench and Python callers can drive it with raw device
pointers (e.g. ``torch.Tensor.data_ptr()``) and HIP stream handles.

Names, argument meaning and error behaviour follow the reference's public API
(/root/reference/src/nccl.h.in): every call returns/raises on the same
``ncclResult_t`` codes. There is NO fallback: if the library is missing or a
symbol is absent, loading raises immediately.

Directory name has a hyphen, so import it through ``load()`` below or
``importlib`` (see tests/conftest.py)::

    nbx = load_package()            # helper in tests / bench
    comm = nbx.Communicator.init_rank(1, nbx.get_unique_id(), 0)
    comm.all_reduce(x.data_ptr(), y.data_ptr(), n, nbx.ncclDataType.ncclFloat32,
                    nbx.ncclRedOp.ncclSum, stream)
"""
from __future__ import annotations

import ctypes
import enum
import os
from typing import Iterable, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libnbxccl.so")
CSRC_DIR = os.path.join(_HERE, "csrc")


class ncclResult(enum.IntEnum):          # nccl.h.in:37-45
    ncclSuccess = 0
    ncclUnhandledCudaError = 1
    ncclSystemError = 2
    ncclInternalError = 3
    ncclInvalidArgument = 4
    ncclInvalidUsage = 5
    ncclRemoteError = 6
    ncclInProgress = 7


class ncclRedOp(enum.IntEnum):           # nccl.h.in:181-197
    ncclSum = 0
    ncclProd = 1
    ncclMax = 2
    ncclMin = 3
    ncclAvg = 4


class ncclDataType(enum.IntEnum):        # nccl.h.in:199-214 (+ fp8, this build)
    ncclInt8 = 0
    ncclUint8 = 1
    ncclInt32 = 2
    ncclUint32 = 3
    ncclInt64 = 4
    ncclUint64 = 5
    ncclFloat16 = 6
    ncclFloat32 = 7
    ncclFloat64 = 8
    ncclBfloat16 = 9
    ncclFloat8e4m3 = 10
    ncclFloat8e5m2 = 11


class ncclScalarResidence(enum.IntEnum):  # nccl.h.in:217-225
    ncclScalarDevice = 0
    ncclScalarHostImmediate = 1


class DevRedOp(enum.IntEnum):            # src/include/device.h:26-30
    Sum = 0
    Prod = 1
    MinMax = 2
    PreMulSum = 3
    SumPostDiv = 4


TYPE_SIZE = {
    ncclDataType.ncclInt8: 1, ncclDataType.ncclUint8: 1,
    ncclDataType.ncclInt32: 4, ncclDataType.ncclUint32: 4,
    ncclDataType.ncclInt64: 8, ncclDataType.ncclUint64: 8,
    ncclDataType.ncclFloat16: 2, ncclDataType.ncclFloat32: 4,
    ncclDataType.ncclFloat64: 8, ncclDataType.ncclBfloat16: 2,
    ncclDataType.ncclFloat8e4m3: 1, ncclDataType.ncclFloat8e5m2: 1,
}

NCCL_UNIQUE_ID_BYTES = 128
NBX_MAX_SRCS = 64
NBX_MAX_DSTS = 8


class ncclUniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * NCCL_UNIQUE_ID_BYTES)]


class DevRedOpFull(ctypes.Structure):    # include/nbx_reduce.h nbxDevRedOpFull
    _fields_ = [("op", ctypes.c_int32), ("scalarArgIsPtr", ctypes.c_int32),
                ("scalarArg", ctypes.c_uint64)]

    def __repr__(self) -> str:
        return (f"DevRedOpFull(op={DevRedOp(self.op).name}, isPtr={bool(self.scalarArgIsPtr)}, "
                f"arg=0x{self.scalarArg:x})")


class NcclError(RuntimeError):
    def __init__(self, code: int, where: str, detail: str = ""):
        self.code = ncclResult(code) if code in ncclResult._value2member_map_ else code
        msg = f"{where} failed: {self.code!r}"
        if detail:
            msg += f" ({detail})"
        super().__init__(msg)


# ---------------------------------------------------------------------------
# Library binding

_lib: Optional[ctypes.CDLL] = None

class ReduceTask(ctypes.Structure):
    """nbxReduceTask (include/nbx_reduce.h): one bucket of nbxReduceMultiBatch."""
    _fields_ = [("dsts", ctypes.POINTER(ctypes.c_void_p)), ("nDsts", ctypes.c_int),
                ("srcs", ctypes.POINTER(ctypes.c_void_p)), ("nSrcs", ctypes.c_int),
                ("count", ctypes.c_size_t)]


_SIGS = {
    # public ABI (include/nccl.h)
    "ncclGetVersion": [ctypes.POINTER(ctypes.c_int)],
    "ncclGetUniqueId": [ctypes.POINTER(ncclUniqueId)],
    "ncclCommInitRank": [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ncclUniqueId, ctypes.c_int],
    "ncclCommInitAll": [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.POINTER(ctypes.c_int)],
    "ncclCommFinalize": [ctypes.c_void_p],
    "ncclCommDestroy": [ctypes.c_void_p],
    "ncclCommAbort": [ctypes.c_void_p],
    "ncclCommSplit": [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p],
    "ncclMemAlloc": [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t],
    "ncclMemFree": [ctypes.c_void_p],
    "ncclCommRegister": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)],
    "ncclCommDeregister": [ctypes.c_void_p, ctypes.c_void_p],
    "ncclCommGetAsyncError": [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)],
    "ncclCommCount": [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)],
    "ncclCommCuDevice": [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)],
    "ncclCommUserRank": [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)],
    "ncclRedOpCreatePreMulSum": [ctypes.POINTER(ctypes.c_int), ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p],
    "ncclRedOpDestroy": [ctypes.c_int, ctypes.c_void_p],
    "ncclReduce": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.c_void_p, ctypes.c_void_p],
    "ncclAllReduce": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                      ctypes.c_void_p, ctypes.c_void_p],
    "ncclReduceScatter": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                          ctypes.c_void_p, ctypes.c_void_p],
    "ncclGroupStart": [],
    "ncclGroupEnd": [],
    # core ABI (include/nbx_reduce.h)
    "nbxHostToDevRedOp": [ctypes.POINTER(DevRedOpFull), ctypes.c_int, ctypes.c_int, ctypes.c_int],
    "nbxReduceMulti": [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                       ctypes.c_int, ctypes.c_size_t, ctypes.c_int, DevRedOpFull, ctypes.c_int, ctypes.c_int,
                       ctypes.c_void_p],
    "nbxReduceMultiHost": [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                           ctypes.c_int, ctypes.c_size_t, ctypes.c_int, DevRedOpFull, ctypes.c_int, ctypes.c_int,
                           ctypes.c_void_p],
    "nbxReduceMultiBatch": [ctypes.POINTER(ReduceTask), ctypes.c_int, ctypes.c_int, DevRedOpFull, ctypes.c_int,
                            ctypes.c_int, ctypes.c_void_p],
    "nbxSetLaunchConfig": [ctypes.c_int, ctypes.c_int],
    "nbxGetLaunchConfig": [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)],
    "nbxKernelCount": [],
    "nbxAbiVersion": [],
}
_RESTYPE_OVERRIDES = {
    "ncclGetErrorString": ctypes.c_char_p,
    "ncclGetLastError": ctypes.c_char_p,
    "nbxKernelCount": ctypes.c_int,
    "nbxAbiVersion": ctypes.c_int,
}

# every symbol the headers declare (checked by tests/test_abi.py)
PUBLIC_SYMBOLS = sorted(set(_SIGS) | {"ncclGetErrorString", "ncclGetLastError", "ncclCommInitRankConfig"})


def library_path() -> str:
    return os.environ.get("NBX_LIB", LIB_PATH)


def load_library(path: Optional[str] = None) -> ctypes.CDLL:
    """Load libnbxccl.so; raise loudly when it is missing (no CPU fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or library_path()
    if not os.path.exists(p):
        raise ImportError(
            f"libnbxccl.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(make -C neuronabox-nccl_amd/csrc). There is no CPU fallback.")
    # One HIP runtime per process: PyTorch-ROCm wheels ship their own
    # libamdhip64 (soname libamdhip64.so.7, loaded by file name). Loading torch
    # first makes libnbxccl's libamdhip64.so.7 dependency resolve to that copy;
    # the other order maps two runtimes and the second sees no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPE_OVERRIDES.get(name, ctypes.c_int)
    for name in ("ncclGetErrorString", "ncclGetLastError"):
        fn = getattr(lib, name)
        fn.restype = ctypes.c_char_p
    lib.ncclGetErrorString.argtypes = [ctypes.c_int]
    lib.ncclGetLastError.argtypes = [ctypes.c_void_p]
    if path is None:
        _lib = lib
    return lib


# Build provenance: build() stamps lib/build_info.json with a digest of the
# sources make built the library from and of the library itself; the bench
# line and smoke() report whether the library on disk is still that build and
# the sources beside it are still those sources (a stale or foreign .so shows).
BUILD_INFO_PATH = os.path.join(_HERE, "lib", "build_info.json")
INCLUDE_DIR = os.path.join(os.path.dirname(_HERE), "include")
_SOURCE_SUFFIXES = (".cc", ".h", ".hip", ".inc")


def _file_sha256(path: str) -> str:
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for block in iter(lambda: f.read(1 << 20), b""):
            h.update(block)
    return h.hexdigest()


def source_digest(csrc_dir: str = CSRC_DIR, include_dir: str = INCLUDE_DIR) -> tuple:
    """(sha256 over every library source by name and content, file count):
    csrc/*.{cc,h,hip,inc}, csrc/Makefile and include/*.h."""
    import hashlib
    files = [("csrc", csrc_dir, f) for f in sorted(os.listdir(csrc_dir))
             if f.endswith(_SOURCE_SUFFIXES) or f == "Makefile"]
    files += [("include", include_dir, f) for f in sorted(os.listdir(include_dir)) if f.endswith(".h")]
    h = hashlib.sha256()
    for tag, d, f in files:
        h.update(f"{tag}/{f}".encode() + b"\0")
        h.update(_file_sha256(os.path.join(d, f)).encode() + b"\n")
    return h.hexdigest(), len(files)


def write_build_info(path: str = BUILD_INFO_PATH) -> dict:
    """Record the digests after a successful make (called by build())."""
    import json
    src, nfiles = source_digest()
    lib = library_path()
    info = {"sources_sha256": src, "source_files": nfiles, "lib_sha256": _file_sha256(lib),
            "lib_bytes": os.path.getsize(lib), "arch": "gfx950"}
    with open(path, "w") as f:
        json.dump(info, f, indent=1)
    return info


def build_info(path: str = BUILD_INFO_PATH) -> dict:
    """The recorded stamp plus two live checks: `lib_matches` (the library on
    disk is the stamped build) and `sources_match` (the sources beside it are
    the ones it was built from). None when no stamp exists."""
    import json
    if not os.path.exists(path):
        return {"recorded": None, "lib_matches": None, "sources_match": None}
    with open(path) as f:
        rec = json.load(f)
    lib = library_path()
    lib_ok = os.path.exists(lib) and _file_sha256(lib) == rec.get("lib_sha256")
    src_ok = source_digest()[0] == rec.get("sources_sha256") if os.path.isdir(CSRC_DIR) else None
    return {"recorded": rec, "lib_matches": lib_ok, "sources_match": src_ok}


def _check(code: int, where: str) -> None:
    if code != ncclResult.ncclSuccess:
        lib = load_library()
        detail = (lib.ncclGetLastError(None) or b"").decode(errors="replace")
        raise NcclError(code, where, detail)


def get_version() -> int:
    v = ctypes.c_int()
    _check(load_library().ncclGetVersion(ctypes.byref(v)), "ncclGetVersion")
    return v.value


def get_error_string(code: int) -> str:
    return load_library().ncclGetErrorString(int(code)).decode()


def get_unique_id() -> ncclUniqueId:
    uid = ncclUniqueId()
    _check(load_library().ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
    return uid


def group_start() -> None:
    _check(load_library().ncclGroupStart(), "ncclGroupStart")


def group_end() -> None:
    _check(load_library().ncclGroupEnd(), "ncclGroupEnd")


def host_to_dev_redop(op: int, dtype: int, nranks: int) -> DevRedOpFull:
    """hostToDevRedOp (enqueue.cc:1436-1512) for the built-in ops."""
    out = DevRedOpFull()
    _check(load_library().nbxHostToDevRedOp(ctypes.byref(out), int(op), int(dtype), int(nranks)),
           "nbxHostToDevRedOp")
    return out


def set_launch_config(blocks_per_cu: int = 0, variant: int = 0) -> None:
    _check(load_library().nbxSetLaunchConfig(int(blocks_per_cu), int(variant)), "nbxSetLaunchConfig")


def get_launch_config() -> tuple:
    b, p = ctypes.c_int(), ctypes.c_int()
    _check(load_library().nbxGetLaunchConfig(ctypes.byref(b), ctypes.byref(p)), "nbxGetLaunchConfig")
    return b.value, p.value


def reduce_multi_raw(dsts: Sequence[int], srcs: Sequence[int], count: int, dtype: int, op: DevRedOpFull,
                     n_pre_op_srcs: int = 0, post_op: bool = False, stream: int = 0) -> int:
    """Call nbxReduceMulti; returns the ncclResult_t code (no raise)."""
    d = (ctypes.c_void_p * max(1, len(dsts)))(*[ctypes.c_void_p(int(x)) for x in dsts])
    s = (ctypes.c_void_p * max(1, len(srcs)))(*[ctypes.c_void_p(int(x)) for x in srcs])
    return load_library().nbxReduceMulti(d, len(dsts), s, len(srcs), int(count), int(dtype), op,
                                         int(n_pre_op_srcs), int(bool(post_op)), ctypes.c_void_p(int(stream)))


def reduce_multi(dsts: Sequence[int], srcs: Sequence[int], count: int, dtype: int, op: DevRedOpFull,
                 n_pre_op_srcs: int = 0, post_op: bool = False, stream: int = 0) -> None:
    """The hot path: ordered left fold of `srcs` into every `dsts` (reduceCopy semantics)."""
    _check(reduce_multi_raw(dsts, srcs, count, dtype, op, n_pre_op_srcs, post_op, stream), "nbxReduceMulti")


def reduce_multi_batch_raw(buckets: Sequence[tuple], dtype: int, op: DevRedOpFull, n_pre_op_srcs: int = 0,
                           post_op: bool = False, stream: int = 0) -> int:
    """Call nbxReduceMultiBatch over buckets [(dsts, srcs, count), ...]; returns the code."""
    keep = []
    tasks = (ReduceTask * max(1, len(buckets)))()
    for i, (dsts, srcs, count) in enumerate(buckets):
        d = (ctypes.c_void_p * max(1, len(dsts)))(*[ctypes.c_void_p(int(x)) for x in dsts])
        s = (ctypes.c_void_p * max(1, len(srcs)))(*[ctypes.c_void_p(int(x)) for x in srcs])
        keep += [d, s]
        tasks[i] = ReduceTask(ctypes.cast(d, ctypes.POINTER(ctypes.c_void_p)), len(dsts),
                              ctypes.cast(s, ctypes.POINTER(ctypes.c_void_p)), len(srcs), int(count))
    return load_library().nbxReduceMultiBatch(tasks, len(buckets), int(dtype), op, int(n_pre_op_srcs),
                                              int(bool(post_op)), ctypes.c_void_p(int(stream)))


def reduce_multi_batch(buckets: Sequence[tuple], dtype: int, op: DevRedOpFull, n_pre_op_srcs: int = 0,
                       post_op: bool = False, stream: int = 0) -> None:
    """Independent buckets [(dsts, srcs, count), ...] reduced as batched launches."""
    _check(reduce_multi_batch_raw(buckets, dtype, op, n_pre_op_srcs, post_op, stream), "nbxReduceMultiBatch")


def reduce_multi_host(dsts: Sequence[int], srcs: Sequence[int], count: int, dtype: int, op: DevRedOpFull,
                      n_pre_op_srcs: int = 0, post_op: bool = False, stream: int = 0) -> None:
    """Host-staged reduction (host pointers in and out; blocking)."""
    d = (ctypes.c_void_p * max(1, len(dsts)))(*[ctypes.c_void_p(int(x)) for x in dsts])
    s = (ctypes.c_void_p * max(1, len(srcs)))(*[ctypes.c_void_p(int(x)) for x in srcs])
    _check(load_library().nbxReduceMultiHost(d, len(dsts), s, len(srcs), int(count), int(dtype), op,
                                             int(n_pre_op_srcs), int(bool(post_op)), ctypes.c_void_p(int(stream))),
           "nbxReduceMultiHost")


class ncclConfig(ctypes.Structure):
    """ncclConfig_t (include/nccl.h; nccl.h.in:53-79), NCCL_CONFIG_INITIALIZER defaults."""
    _fields_ = [("size", ctypes.c_size_t), ("magic", ctypes.c_uint), ("version", ctypes.c_uint),
                ("blocking", ctypes.c_int), ("cgaClusterSize", ctypes.c_int), ("minCTAs", ctypes.c_int),
                ("maxCTAs", ctypes.c_int), ("netName", ctypes.c_char_p), ("splitShare", ctypes.c_int)]

    UNDEF_INT = -(2 ** 31)

    @classmethod
    def initializer(cls, blocking: int | None = None, **fields) -> "ncclConfig":
        """NCCL_CONFIG_INITIALIZER, then `blocking` and any other field by name
        (minCTAs, maxCTAs, cgaClusterSize, splitShare, ...)."""
        c = cls(ctypes.sizeof(cls), 0xcafebeef, 21904, cls.UNDEF_INT, cls.UNDEF_INT, cls.UNDEF_INT, cls.UNDEF_INT,
                None, cls.UNDEF_INT)
        if blocking is not None:
            c.blocking = int(blocking)
        for k, v in fields.items():
            setattr(c, k, v)
        return c


class Communicator:
    """ncclComm_t wrapper (lifecycle + reducing collectives)."""

    def __init__(self, handle: int):
        self.handle = ctypes.c_void_p(handle)

    @classmethod
    def init_rank(cls, nranks: int, uid: ncclUniqueId, rank: int) -> "Communicator":
        h = ctypes.c_void_p()
        _check(load_library().ncclCommInitRank(ctypes.byref(h), int(nranks), uid, int(rank)), "ncclCommInitRank")
        return cls(h.value)

    @classmethod
    def init_rank_config(cls, nranks: int, uid: ncclUniqueId, rank: int, blocking: int | None = None, **fields):
        """ncclCommInitRankConfig; returns (communicator, result code). A
        non-blocking communicator (blocking=0) comes back at once with
        ncclInProgress; poll async_error() until it is no longer ncclInProgress.
        Other ncclConfig_t fields by name (minCTAs=..., maxCTAs=...)."""
        h = ctypes.c_void_p()
        cfg = ncclConfig.initializer(blocking, **fields)
        rc = load_library().ncclCommInitRankConfig(ctypes.byref(h), int(nranks), uid, int(rank), ctypes.byref(cfg))
        if rc not in (ncclResult.ncclSuccess, ncclResult.ncclInProgress):
            _check(rc, "ncclCommInitRankConfig")
        return cls(h.value), int(rc)

    @classmethod
    def init_all(cls, devices: Iterable[int]) -> list:
        devs = list(devices)
        hs = (ctypes.c_void_p * len(devs))()
        dl = (ctypes.c_int * len(devs))(*devs)
        _check(load_library().ncclCommInitAll(hs, len(devs), dl), "ncclCommInitAll")
        return [cls(hs[i]) for i in range(len(devs))]

    def count(self) -> int:
        v = ctypes.c_int()
        _check(load_library().ncclCommCount(self.handle, ctypes.byref(v)), "ncclCommCount")
        return v.value

    def device(self) -> int:
        v = ctypes.c_int()
        _check(load_library().ncclCommCuDevice(self.handle, ctypes.byref(v)), "ncclCommCuDevice")
        return v.value

    def user_rank(self) -> int:
        v = ctypes.c_int()
        _check(load_library().ncclCommUserRank(self.handle, ctypes.byref(v)), "ncclCommUserRank")
        return v.value

    def async_error(self) -> int:
        v = ctypes.c_int()
        _check(load_library().ncclCommGetAsyncError(self.handle, ctypes.byref(v)), "ncclCommGetAsyncError")
        return v.value

    def all_reduce(self, send: int, recv: int, count: int, dtype: int, op: int, stream: int = 0) -> None:
        _check(load_library().ncclAllReduce(ctypes.c_void_p(send), ctypes.c_void_p(recv), int(count), int(dtype),
                                            int(op), self.handle, ctypes.c_void_p(stream)), "ncclAllReduce")

    def reduce_scatter(self, send: int, recv: int, recvcount: int, dtype: int, op: int, stream: int = 0) -> None:
        _check(load_library().ncclReduceScatter(ctypes.c_void_p(send), ctypes.c_void_p(recv), int(recvcount),
                                                int(dtype), int(op), self.handle, ctypes.c_void_p(stream)),
               "ncclReduceScatter")

    def reduce(self, send: int, recv: int, count: int, dtype: int, op: int, root: int, stream: int = 0) -> None:
        _check(load_library().ncclReduce(ctypes.c_void_p(send), ctypes.c_void_p(recv), int(count), int(dtype),
                                         int(op), int(root), self.handle, ctypes.c_void_p(stream)), "ncclReduce")

    def redop_create_premulsum(self, scalar_ptr: int, dtype: int,
                               residence: int = ncclScalarResidence.ncclScalarHostImmediate) -> int:
        op = ctypes.c_int()
        _check(load_library().ncclRedOpCreatePreMulSum(ctypes.byref(op), ctypes.c_void_p(scalar_ptr), int(dtype),
                                                       int(residence), self.handle), "ncclRedOpCreatePreMulSum")
        return op.value

    def redop_destroy(self, op: int) -> None:
        _check(load_library().ncclRedOpDestroy(int(op), self.handle), "ncclRedOpDestroy")

    def finalize(self) -> None:
        _check(load_library().ncclCommFinalize(self.handle), "ncclCommFinalize")

    def split(self, color: int, key: int, blocking: int | None = None):
        """ncclCommSplit (collective over this communicator); returns (child or
        None for NCCL_SPLIT_NOCOLOR, result code)."""
        h = ctypes.c_void_p()
        cfg = ncclConfig.initializer(blocking) if blocking is not None else None
        rc = load_library().ncclCommSplit(self.handle, int(color), int(key), ctypes.byref(h),
                                          ctypes.cast(ctypes.pointer(cfg), ctypes.c_void_p) if cfg is not None else None)
        if rc not in (ncclResult.ncclSuccess, ncclResult.ncclInProgress):
            _check(rc, "ncclCommSplit")
        return (Communicator(h.value) if h.value else None), int(rc)

    def register(self, ptr: int, size: int) -> int:
        """ncclCommRegister; returns the registration handle."""
        h = ctypes.c_void_p()
        _check(load_library().ncclCommRegister(self.handle, ctypes.c_void_p(ptr), int(size), ctypes.byref(h)),
               "ncclCommRegister")
        return h.value

    def deregister(self, handle: int) -> None:
        _check(load_library().ncclCommDeregister(self.handle, ctypes.c_void_p(handle)), "ncclCommDeregister")

    def destroy(self) -> None:
        if self.handle:
            _check(load_library().ncclCommDestroy(self.handle), "ncclCommDestroy")
            self.handle = ctypes.c_void_p()

    def abort(self) -> None:
        """ncclCommAbort: ends every spinning wait of this communicator, frees it."""
        if self.handle:
            _check(load_library().ncclCommAbort(self.handle), "ncclCommAbort")
            self.handle = ctypes.c_void_p()


# ---------------------------------------------------------------------------
# torch helpers (torch is plumbing only: device memory and streams)

def torch_dtype_to_nccl(dt) -> ncclDataType:
    import torch
    table = {
        torch.int8: ncclDataType.ncclInt8, torch.uint8: ncclDataType.ncclUint8,
        torch.int32: ncclDataType.ncclInt32, torch.int64: ncclDataType.ncclInt64,
        torch.float16: ncclDataType.ncclFloat16, torch.float32: ncclDataType.ncclFloat32,
        torch.float64: ncclDataType.ncclFloat64, torch.bfloat16: ncclDataType.ncclBfloat16,
        torch.float8_e4m3fn: ncclDataType.ncclFloat8e4m3, torch.float8_e5m2: ncclDataType.ncclFloat8e5m2,
    }
    for k in ("uint32", "uint64"):
        if hasattr(torch, k):
            table[getattr(torch, k)] = ncclDataType[f"ncclUint{k[4:]}"]
    return table[dt]


def current_stream_handle() -> int:
    import torch
    return int(torch.cuda.current_stream().cuda_stream)
