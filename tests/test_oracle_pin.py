"""Pin the CPU oracle before trusting it (CPU-only).

1. Known answers SURVEY.md §8(c) recorded from the reference's own functors
   (tests/golden/survey_known_answers.json).
2. hostToDevRedOp encodings transcribed from enqueue.cc:1457-1499.
3. Independent cross-checks of the arithmetic: numpy IEEE / modular ops in
   the same left-fold order (f32, f64, integers), numpy/torch dtype casts for
   the f16 / bf16 / fp8 codecs.
"""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "survey_known_answers.json")


def _h(x):
    return int(x, 16)


def _load():
    with open(GOLD) as f:
        return json.load(f)


@pytest.mark.parametrize("case", _load()["reduce"], ids=lambda c: c["name"])
def test_known_answers(oracle, case):
    dt = case["dtype"]
    st = oracle.NP_STORAGE[dt]
    ut = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[np.dtype(st).itemsize]
    srcs = [np.array([_h(v) for v in s], dtype=ut).view(st) for s in case["srcs"]]
    out = oracle.reduce_multi(srcs, dt, case["devop"], _h(case["arg"]), case.get("npre", 0),
                              bool(case.get("postop", 0)))[0]
    assert [int(x) for x in out.view(ut)] == [_h(v) for v in case["expect"]]


@pytest.mark.parametrize("case", _load()["redop"], ids=lambda c: c["why"])
def test_redop_encoding(oracle, case):
    devop, arg = oracle.host_to_dev_redop(case["op"], case["dtype"], case["nranks"])
    assert devop == case["devop"]
    assert arg == _h(case["arg"])


def _fold_numpy(srcs, fn):
    acc = srcs[0].copy()
    for s in srcs[1:]:
        acc = fn(acc, s)
    return acc


@pytest.mark.parametrize("dtype", [7, 8])
@pytest.mark.parametrize("devop", [0, 1])
@pytest.mark.parametrize("nsrc", [2, 5, 8])
def test_float_fold_matches_numpy(oracle, dtype, devop, nsrc):
    srcs = oracle.random_inputs(dtype, nsrc, 10007, seed=11, specials=True)
    got = oracle.reduce_multi(srcs, dtype, devop, threads=3)[0]
    with np.errstate(all="ignore"):
        ref = _fold_numpy(srcs, np.add if devop == 0 else np.multiply)
    np.testing.assert_array_equal(got.view(np.uint8)[~np.isnan(np.repeat(ref, ref.itemsize))],
                                  ref.view(np.uint8)[~np.isnan(np.repeat(ref, ref.itemsize))])
    assert np.array_equal(np.isnan(got), np.isnan(ref))


@pytest.mark.parametrize("dtype", [7, 8])
@pytest.mark.parametrize("is_max", [False, True])
def test_float_minmax_rule(oracle, dtype, is_max):
    st = oracle.NP_STORAGE[dtype]
    a = np.array([1.0, np.nan, 2.0, np.nan, 0.0, -0.0, 5.0, -3.0], dtype=st)
    b = np.array([np.nan, 1.0, np.nan, np.nan, -0.0, 0.0, 5.0, -4.0], dtype=st)
    arg = 0xFFFFFFFF if (is_max and dtype == 7) else (0xFFFFFFFFFFFFFFFF if is_max else 0)
    got = oracle.reduce_multi([a, b], dtype, 2, arg)[0]
    exp = np.array([1.0, 1.0, 2.0, np.nan, -0.0, 0.0, 5.0, -3.0 if is_max else -4.0], dtype=st)
    # NaN operand -> other operand; tie (incl. +-0) -> second operand
    assert np.array_equal(np.isnan(got), np.isnan(exp))
    m = ~np.isnan(exp)
    assert np.array_equal(np.signbit(got[m]), np.signbit(exp[m]))
    np.testing.assert_array_equal(got[m], exp[m])


@pytest.mark.parametrize("dtype", [0, 1, 2, 3, 4, 5])
def test_integer_ops_match_numpy(oracle, dtype):
    st = oracle.NP_STORAGE[dtype]
    srcs = oracle.random_inputs(dtype, 4, 4099, seed=5)
    u = {1: np.uint8, 4: np.uint32, 8: np.uint64}[np.dtype(st).itemsize]
    us = [s.view(u) for s in srcs]
    with np.errstate(all="ignore"):
        np.testing.assert_array_equal(oracle.reduce_multi(srcs, dtype, 0)[0].view(u), _fold_numpy(us, np.add))
        np.testing.assert_array_equal(oracle.reduce_multi(srcs, dtype, 1)[0].view(u), _fold_numpy(us, np.multiply))
    for op in (2, 3):   # ncclMax, ncclMin via hostToDevRedOp xormask
        devop, arg = oracle.host_to_dev_redop(op, dtype, 1)
        got = oracle.reduce_multi(srcs, dtype, devop, arg)[0]
        exp = _fold_numpy(srcs, np.maximum if op == 2 else np.minimum)
        np.testing.assert_array_equal(got, exp)
    # Avg on integers: SumPostDiv with C truncating division of the wrapped sum
    devop, arg = oracle.host_to_dev_redop(4, dtype, 4)
    got = oracle.reduce_multi(srcs, dtype, devop, arg, post_op=True)[0]
    with np.errstate(all="ignore"):
        wsum = _fold_numpy(us, np.add).view(st)
    if np.issubdtype(st, np.signedinteger):
        # C division truncates toward zero
        exp = np.array([(abs(int(x)) // 4) * (1 if x >= 0 else -1) for x in wsum], dtype=np.int64).astype(st)
    else:
        exp = wsum // 4
    np.testing.assert_array_equal(got, exp)


def test_premulsum_pre_op_only_on_first_sources(oracle):
    srcs = [np.full(8, 3.0, np.float32), np.full(8, 5.0, np.float32), np.full(8, 7.0, np.float32)]
    scal = int(np.float32(0.5).view(np.uint32))
    got = oracle.reduce_multi(srcs, 7, 3, scal, n_pre_op_srcs=2)[0]
    np.testing.assert_array_equal(got, np.full(8, 3.0 * 0.5 + 5.0 * 0.5 + 7.0, np.float32))


def test_f16_codec_matches_numpy_exhaustive(oracle):
    codes = np.arange(65536, dtype=np.uint16)
    ref = codes.view(np.float16).astype(np.float32)
    got = np.array([oracle.f16_to_f32(int(c)) for c in codes], dtype=np.float32)
    m = ~np.isnan(ref)
    np.testing.assert_array_equal(got[m], ref[m])
    assert np.isnan(got[~m]).all()
    rng = np.random.default_rng(3)
    f = np.concatenate([rng.standard_normal(20000).astype(np.float32) * 10 ** rng.uniform(-9, 5, 20000).astype(np.float32),
                        ref[m][::7], np.float32([65504, 65519.99, 65520, 7e4, 1e-8, 3e-8, 2.98e-8])])
    got = np.array([oracle.f32_to_f16(float(x)) for x in f], dtype=np.uint16)
    np.testing.assert_array_equal(got, f.astype(np.float16).view(np.uint16))


def test_bf16_codec_matches_torch(oracle):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(4)
    f = np.concatenate([rng.standard_normal(20000).astype(np.float32) * 10 ** rng.uniform(-38, 38, 20000).astype(np.float32),
                        np.float32([1e-40, -3e-39, 3.39e38, 3.4e38, np.inf, -np.inf, 0.0, -0.0])])
    got = np.array([oracle.f32_to_bf16(float(x)) for x in f], dtype=np.uint16)
    ref = torch.from_numpy(f).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("dtype", [10, 11])
def test_fp8_codec_matches_torch(oracle, dtype):
    """fp8 is this build's extension (parity unpinned vs the reference); the
    codec itself is checked against torch's OCP float8 types, with SATFINITE
    (finite values beyond the largest code clamped to it before torch's cast,
    inf and NaN passed as they are — HIP's amd_hip_fp8.h definition, which
    RCCL's fp8 functors use)."""
    torch = pytest.importorskip("torch")
    tdt = torch.float8_e4m3fn if dtype == 10 else torch.float8_e5m2
    dec = oracle.e4m3_to_f32 if dtype == 10 else oracle.e5m2_to_f32
    enc = oracle.f32_to_e4m3 if dtype == 10 else oracle.f32_to_e5m2
    codes = np.arange(256, dtype=np.uint8)
    ref = torch.from_numpy(codes).view(tdt).to(torch.float32).numpy()
    got = np.array([dec(int(c)) for c in codes], dtype=np.float32)
    m = ~np.isnan(ref)
    np.testing.assert_array_equal(got[m], ref[m])
    assert np.isnan(got[~m]).all()
    rng = np.random.default_rng(9)
    mx = 448.0 if dtype == 10 else 57344.0
    f = np.concatenate([rng.uniform(-1.2 * mx, 1.2 * mx, 20000).astype(np.float32),
                        (rng.standard_normal(20000) * 10 ** rng.uniform(-9, 0, 20000)).astype(np.float32),
                        ref[m], (ref[m][:-1] + np.diff(ref[m]) / 2).astype(np.float32)])
    f = np.concatenate([f, np.float32([mx * 1.01, -mx * 1.5, 1e30, -3e38, np.inf, -np.inf, np.nan])])
    got = np.array([enc(float(x)) for x in f], dtype=np.uint8)
    sat = np.where(np.isfinite(f), np.clip(f, -mx, mx), f).astype(np.float32)
    tref = torch.from_numpy(sat).to(tdt).view(torch.uint8).numpy()
    gnan = np.isnan(np.array([dec(int(c)) for c in got]))
    rnan = np.isnan(torch.from_numpy(tref).view(tdt).to(torch.float32).numpy())
    assert np.array_equal(gnan, rnan)
    np.testing.assert_array_equal(got[~gnan], tref[~gnan])
