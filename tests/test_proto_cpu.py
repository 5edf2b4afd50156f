"""Protocol selection of the multi-process communicator, on the CPU through
the library's debug hooks (include/nbx_debug.h): NCCL_PROTO parsing in NCCL's
list syntax (tuning.cc:254-259: "LL,LL128", "^Simple", case-insensitive) and
the per-message choice LL (<= LL max) -> LL128 (<= LL128 max, <= 8 ranks):
one-shot (AllReduce with > 2 ranks only up to the one-shot max), else two-shot
AllReduce / Reduce (a rank's block fits half an LL128 slot) -> Simple;
ReduceScatter (one hop by nature) one-shot up to the LL128 max."""
import ctypes

import pytest

LL, LL128, SIMPLE, ALL = 1, 2, 4, 7
P_LL, P_LL128, P_SIMPLE = 0, 1, 2


@pytest.fixture(scope="module")
def lib(nbx):
    lib = nbx.load_library()
    lib.nbxDebugProtoMask.argtypes = [ctypes.c_char_p]
    lib.nbxDebugProtoMask.restype = ctypes.c_int
    lib.nbxDebugChooseProto.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                        ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
    lib.nbxDebugChooseProto.restype = ctypes.c_int
    return lib


@pytest.mark.parametrize("s,mask", [
    (None, ALL), ("", ALL), ("LL", LL), ("ll128", LL128), ("Simple", SIMPLE), ("LL,Simple", LL | SIMPLE),
    ("LL128,LL", LL | LL128), ("^LL128", LL | SIMPLE), ("^ll,simple", LL128), ("^", ALL), ("LL,,Simple", LL | SIMPLE),
    ("bogus", 0), ("LL,bogus", LL),
])
def test_nccl_proto_parsing(lib, s, mask):
    assert lib.nbxDebugProtoMask(None if s is None else s.encode()) == mask


K, M = 1 << 10, 1 << 20
P_LL128X2 = 3


def _block(nbytes, n, eb=4):
    epp = 16 // eb
    per = -(-(nbytes // eb) // n)
    return (-(-per // epp) * epp) * eb


@pytest.mark.parametrize("mask,ar,nbytes,n,want", [
    (ALL, 1, 4, 2, P_LL), (ALL, 1, 64 * K, 8, P_LL), (ALL, 1, 64 * K + 4, 8, P_LL128), (ALL, 1, 256 * K, 8, P_LL128),
    (ALL, 1, 256 * K + 4, 8, P_LL128X2), (ALL, 1, 4 * M, 8, P_LL128X2), (ALL, 1, 4 * M + 1024, 8, P_SIMPLE),
    (ALL, 1, 4 * M, 2, P_LL128), (ALL, 1, 4 * M + 4, 2, P_SIMPLE),      # 2 ranks: one-shot only
    (ALL, 1, 4 * M, 3, P_LL128X2), (ALL, 1, 6 * M, 3, P_SIMPLE),      # the slot bounds both shapes
    (ALL, 0, 4 * M, 8, P_LL128), (ALL, 0, 4 * M + 4, 8, P_SIMPLE),      # RS: one-shot up to the max
    (ALL, 1, 256 * K, 9, P_SIMPLE), (ALL, 1, 4 * K, 9, P_LL),           # LL128 only up to 8 ranks
    (ALL, 1, 0, 4, P_SIMPLE), (ALL, 1, 4 * K, 65, P_SIMPLE),
    (LL | SIMPLE, 1, 256 * K, 4, P_SIMPLE), (LL128 | SIMPLE, 1, 4, 4, P_LL128), (SIMPLE, 1, 4, 4, P_SIMPLE),
    (LL, 1, 256 * K, 4, P_SIMPLE),                                       # nothing enabled fits: Simple
])
def test_protocol_choice(lib, mask, ar, nbytes, n, want):
    assert lib.nbxDebugChooseProto(mask, ar, nbytes, _block(nbytes, n), n, 64 * K, 4 * M, 256 * K) == want


def test_ll128_disabled_by_zero_max(lib):
    assert lib.nbxDebugChooseProto(ALL, 1, 256 * K, 64 * K, 4, 64 * K, 0, 256 * K) == P_SIMPLE


# LL128 across GPUs (tuning.cc:250-297: LL128 is "default"
# (2) unless NCCL_PROTO lists it, and default LL128 is enabled only on
# validated fabrics): ranks on distinct GPUs start without LL128 unless
# NCCL_PROTO names it (not in a "^list") or NBX_LL128_ACROSS_GPUS=1; ranks
# sharing a GPU keep it (stress-tested there).
@pytest.mark.parametrize("s,multi,mask", [
    (None, 0, ALL), (None, 1, LL | SIMPLE), ("", 1, LL | SIMPLE),
    ("LL128", 1, LL128), ("LL,LL128", 1, LL | LL128), ("^Simple", 1, LL), ("^LL", 1, SIMPLE),
    ("^Simple", 0, LL | LL128), ("Simple", 1, SIMPLE),
])
def test_ll128_gated_across_gpus(lib, monkeypatch, s, multi, mask):
    monkeypatch.delenv("NBX_LL128_ACROSS_GPUS", raising=False)
    monkeypatch.delenv("NBX_DEBUG_ASSUME_MULTI_GPU", raising=False)
    lib.nbxDebugGatedProtoMask.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.nbxDebugGatedProtoMask.restype = ctypes.c_int
    assert lib.nbxDebugGatedProtoMask(None if s is None else s.encode(), multi) == mask


def test_ll128_across_gpus_overrides(lib, monkeypatch):
    lib.nbxDebugGatedProtoMask.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.nbxDebugGatedProtoMask.restype = ctypes.c_int
    monkeypatch.delenv("NBX_DEBUG_ASSUME_MULTI_GPU", raising=False)
    monkeypatch.setenv("NBX_LL128_ACROSS_GPUS", "1")
    assert lib.nbxDebugGatedProtoMask(None, 1) == ALL
    monkeypatch.setenv("NBX_LL128_ACROSS_GPUS", "0")
    assert lib.nbxDebugGatedProtoMask(None, 1) == LL | SIMPLE
    # the test hook: ranks that share a GPU are gated as if they did not
    monkeypatch.setenv("NBX_DEBUG_ASSUME_MULTI_GPU", "1")
    assert lib.nbxDebugGatedProtoMask(None, 0) == LL | SIMPLE
