"""CPU ORACLE — test infrastructure only (never imported by the product path).

Python/numpy face of oracle/reduce_oracle.c, the plain-C restatement of the
reference's reduction semantics (see that file's header for the line-by-line
citations and the pin status). Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.

PARITY PIN STATUS: partial. The reference (NCCL 2.19.4 device headers) cannot
be compiled here without stand-in CUDA headers, and it ships no tests or
golden vectors; the oracle is pinned against the known-answer values that
SURVEY.md §8c records from the reference's own functors
(tests/golden/survey_known_answers.json) plus independent cross-checks.
fp8 results are "parity unpinned" (the reference has no fp8 type).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

# ncclDataType_t -> numpy storage dtype (raw bit patterns for 16-bit floats / fp8)
NP_STORAGE = {
    0: np.int8, 1: np.uint8, 2: np.int32, 3: np.uint32, 4: np.int64, 5: np.uint64,
    6: np.uint16, 7: np.float32, 8: np.float64, 9: np.uint16, 10: np.uint8, 11: np.uint8,
}
FLOAT_TYPES = {6, 7, 8, 9, 10, 11}
TYPE_NAMES = {0: "int8", 1: "uint8", 2: "int32", 3: "uint32", 4: "int64", 5: "uint64", 6: "float16",
              7: "float32", 8: "float64", 9: "bfloat16", 10: "fp8e4m3", 11: "fp8e5m2"}

_lib: Optional[ctypes.CDLL] = None


def build() -> str:
    """Compile the oracle (gcc) if needed; returns the .so path."""
    src = os.path.join(_HERE, "reduce_oracle.c")
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-C", _HERE], check=True, stdout=subprocess.DEVNULL)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_reduce_multi.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_size_t,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int]
        L.oracle_reduce_multi.restype = ctypes.c_int
        L.oracle_host_to_dev_redop.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_host_to_dev_redop.restype = ctypes.c_int
        L.oracle_type_size.argtypes = [ctypes.c_int]
        for n, a, r in (("oracle_f16_to_f32", ctypes.c_uint16, ctypes.c_float),
                        ("oracle_f32_to_f16", ctypes.c_float, ctypes.c_uint16),
                        ("oracle_bf16_to_f32", ctypes.c_uint16, ctypes.c_float),
                        ("oracle_f32_to_bf16", ctypes.c_float, ctypes.c_uint16),
                        ("oracle_e4m3_to_f32", ctypes.c_uint8, ctypes.c_float),
                        ("oracle_f32_to_e4m3", ctypes.c_float, ctypes.c_uint8),
                        ("oracle_e5m2_to_f32", ctypes.c_uint8, ctypes.c_float),
                        ("oracle_f32_to_e5m2", ctypes.c_float, ctypes.c_uint8)):
            f = getattr(L, n)
            f.argtypes = [a]
            f.restype = r
        _lib = L
    return _lib


def reduce_multi(srcs: Sequence[np.ndarray], dtype: int, devop: int, arg: int = 0, n_pre_op_srcs: int = 0,
                 post_op: bool = False, n_dsts: int = 1, threads: int = 1,
                 out: Optional[Sequence[np.ndarray]] = None) -> list:
    """Reference semantics of reduceCopy over host arrays; returns the n_dsts outputs."""
    st = NP_STORAGE[dtype]
    srcs = [np.ascontiguousarray(s) for s in srcs]
    count = srcs[0].size
    for s in srcs:
        assert s.dtype == np.dtype(st) and s.size == count, (s.dtype, st, s.size, count)
    outs = list(out) if out is not None else [np.empty(count, dtype=st) for _ in range(n_dsts)]
    sp = (ctypes.c_void_p * len(srcs))(*[s.ctypes.data for s in srcs])
    dp = (ctypes.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
    rc = lib().oracle_reduce_multi(dp, len(outs), sp, len(srcs), count, int(dtype), int(devop),
                                   ctypes.c_uint64(int(arg) & 0xFFFFFFFFFFFFFFFF), int(n_pre_op_srcs),
                                   int(bool(post_op)), int(threads))
    if rc != 0:
        raise ValueError(f"oracle_reduce_multi rejected arguments (dtype={dtype}, op={devop}, arg={arg})")
    return outs


def host_to_dev_redop(op: int, dtype: int, nranks: int):
    d = ctypes.c_int()
    a = ctypes.c_uint64()
    rc = lib().oracle_host_to_dev_redop(int(op), int(dtype), int(nranks), ctypes.byref(d), ctypes.byref(a))
    if rc != 0:
        raise ValueError("invalid op/type")
    return d.value, a.value


# scalar codecs (for fixtures / tests)
def f16_to_f32(h: int) -> float: return lib().oracle_f16_to_f32(h)
def f32_to_f16(f: float) -> int: return lib().oracle_f32_to_f16(f)
def bf16_to_f32(h: int) -> float: return lib().oracle_bf16_to_f32(h)
def f32_to_bf16(f: float) -> int: return lib().oracle_f32_to_bf16(f)
def e4m3_to_f32(c: int) -> float: return lib().oracle_e4m3_to_f32(c)
def f32_to_e4m3(f: float) -> int: return lib().oracle_f32_to_e4m3(f)
def e5m2_to_f32(c: int) -> float: return lib().oracle_e5m2_to_f32(c)
def f32_to_e5m2(f: float) -> int: return lib().oracle_f32_to_e5m2(f)


def random_inputs(dtype: int, n_srcs: int, count: int, seed: int, specials: bool = False) -> list:
    """Seeded inputs as raw storage arrays. Floats: uniform[-1,1) RNE-converted
     with optional special values (+-0, denormals, +-inf, NaN);
    integers: full-range random bits."""
    out = []
    for s in range(n_srcs):
        rng = np.random.default_rng(seed + s)
        st = NP_STORAGE[dtype]
        if dtype in (7, 8):
            a = rng.uniform(-1.0, 1.0, count).astype(st)
            if specials and count >= 16:
                sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40 if dtype == 7 else 1e-310,
                               -1e-40 if dtype == 7 else -1e-310, 3.4e38 if dtype == 7 else 1.7e308], dtype=st)
                idx = rng.choice(count, size=min(count // 4, 64), replace=False)
                a[idx] = sp[rng.integers(0, len(sp), idx.size)]
        elif dtype in (6, 9):
            f = rng.uniform(-1.0, 1.0, count).astype(np.float32)
            conv = f32_to_f16 if dtype == 6 else f32_to_bf16
            a = np.fromiter((conv(float(x)) for x in f), dtype=np.uint16, count=count) if count < 200000 else \
                _vec_narrow16(f, dtype)
            if specials and count >= 16:
                sp = np.array([0x0000, 0x8000, 0x0001, 0x8001, 0x7c00 if dtype == 6 else 0x7f80,
                               0xfc00 if dtype == 6 else 0xff80, 0x7e00 if dtype == 6 else 0x7fc0,
                               0x7bff if dtype == 6 else 0x7f7f], dtype=np.uint16)
                idx = rng.choice(count, size=min(count // 4, 64), replace=False)
                a[idx] = sp[rng.integers(0, len(sp), idx.size)]
        elif dtype in (10, 11):
            a = rng.integers(0, 256, count, dtype=np.uint8)
            if not specials:   # finite codes only
                bad = (a & 0x7F) == 0x7F if dtype == 10 else (a & 0x7C) == 0x7C
                a[bad] &= 0xF7 if dtype == 10 else 0xBB
        else:
            info = np.iinfo(st)
            a = rng.integers(info.min, info.max, count, dtype=st, endpoint=True)
        out.append(a)
    return out


def _vec_narrow16(f: np.ndarray, dtype: int) -> np.ndarray:
    """Vectorised RNE fp32 -> f16 / bf16 (same rounding as the C codecs)."""
    if dtype == 6:
        return f.astype(np.float16).view(np.uint16)
    u = f.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = np.isnan(f)
    r[nan] = ((f.view(np.uint32)[nan] >> 16) | 0x40).astype(np.uint16)
    return r
