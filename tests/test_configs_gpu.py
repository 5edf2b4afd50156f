"""BASELINE configs C, D and E at their stated sizes, on the one GPU of the test
box, checked against the CPU oracle ("next round" item 1).

* C — fp16 and bf16 ncclSum, 1..64 MiB per input, nSrcs 2 and 8: single
  buckets through nbxReduceMulti at 32 and 64 MiB, and the whole sweep
  1, 2, 4, ..., 64 MiB through one nbxReduceMultiBatch call (default launch
  policy and launch variant 1, which puts every bucket in the batch kernel).
* D — 8 ranks x 1 GiB fp32 (268,435,456 elements): ncclAllReduce and
  ncclReduceScatter on the multi-process communicator, direct and ring
  schedules (NCCL_ALGO=Ring).
* E — 8 ranks, 128 MiB: ncclAllReduce int64 ncclMax (16,777,216 elements,
  full-range random bits) and fp8 e4m3 ncclSum (134,217,728 elements, random
  finite codes).

The 8 ranks are 8 processes sharing the one GPU (the box has one), so this is
the data path and the schedules at full size — not xGMI. The oracle folds
every block in the schedule's order: AllReduce chunk c and ReduceScatter block
c in ring order c+1, ..., c (all_reduce.h:60-79, reduce_scatter.h:49-64).
Outputs are compared through SHA-256 digests of the whole buffer, every rank.
"""
import hashlib
import multiprocessing as mp
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

F16, BF16, F32, I64, E4M3 = 6, 9, 7, 4, 10


def _say(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


# ----------------------------------------------------------------------------
# config C

def _gpu_half_inputs(torch, dtype, nsrc, count, seed):
    """uniform[-1,1) fp32 RNE-narrowed to fp16 / bf16 on the GPU (torch's casts
    are RNE), returned as uint16 device tensors."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    tdt = torch.float16 if dtype == F16 else torch.bfloat16
    return [(torch.rand(count, device="cuda", generator=g) * 2 - 1).to(tdt).view(torch.int16) for _ in range(nsrc)]


@pytest.mark.parametrize("dtype", [F16, BF16])
@pytest.mark.parametrize("nsrc", [2, 8])
@pytest.mark.parametrize("mib", [32, 64])
def test_config_c_single_bucket(nbx, oracle, torch_gpu, dtype, nsrc, mib):
    torch = torch_gpu
    count = (mib << 20) // 2
    ts = _gpu_half_inputs(torch, dtype, nsrc, count, seed=mib * 100 + nsrc)
    out = torch.empty_like(ts[0])
    op = nbx.DevRedOpFull()
    nbx.reduce_multi([out.data_ptr()], [t.data_ptr() for t in ts], count, dtype, op, 0, False,
                     torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    host = [t.cpu().numpy().view(np.uint16) for t in ts]
    exp = oracle.reduce_multi(host, dtype, 0, threads=16)[0]
    got = out.cpu().numpy().view(np.uint16)
    assert np.array_equal(got, exp), f"{np.count_nonzero(got != exp)} mismatches"


@pytest.mark.parametrize("dtype", [F16, BF16])
@pytest.mark.parametrize("nsrc", [2, 8])
def test_config_c_bucket_sweep_one_batch(nbx, oracle, torch_gpu, dtype, nsrc):
    """The whole config-C sweep (1, 2, 4, ..., 64 MiB per input) as ONE
    nbxReduceMultiBatch call, with the default launch policy (buckets that fill
    the GPU alone take the big-tile kernel) and with launch variant 1 (every
    bucket in the batch kernel)."""
    torch = torch_gpu
    sizes = [1, 2, 4, 8, 16, 32, 64]
    buckets = []
    for k, mib in enumerate(sizes):
        count = (mib << 20) // 2 + (k * 3 if k % 2 else 0)   # some counts not a multiple of 8 elements
        ts = _gpu_half_inputs(torch, dtype, nsrc, count, seed=7000 + 10 * k + nsrc)
        buckets.append((ts, torch.empty_like(ts[0]), count))
    host = [[t.cpu().numpy().view(np.uint16) for t in ts] for ts, _, _ in buckets]
    exps = [oracle.reduce_multi(h, dtype, 0, threads=16)[0] for h in host]
    op = nbx.DevRedOpFull()
    stream = torch.cuda.current_stream().cuda_stream
    try:
        for variant in (0, 1):
            nbx.set_launch_config(0, variant)
            for _, o, _ in buckets:
                o.fill_(0x5A5A)
            nbx.reduce_multi_batch([([o.data_ptr()], [t.data_ptr() for t in ts], c) for ts, o, c in buckets],
                                   dtype, op, 0, False, stream)
            torch.cuda.synchronize()
            for (ts, o, c), e, mib in zip(buckets, exps, sizes):
                got = o.cpu().numpy().view(np.uint16)
                assert np.array_equal(got, e), f"variant {variant}, {mib} MiB: {np.count_nonzero(got != e)} mismatches"
    finally:
        nbx.set_launch_config(0, 0)


# ----------------------------------------------------------------------------
# configs D and E: 8 processes, one per rank

N_RANKS = 8
COUNT_D = 256 << 20          # fp32 elements per rank (1 GiB)
RC_D = COUNT_D // N_RANKS    # ReduceScatter recvcount (128 MiB per rank)
COUNT_E_I64 = 16 << 20       # 128 MiB of int64
COUNT_E_F8 = 128 << 20       # 128 MiB of fp8 e4m3


def _input_d(r):
    x = np.random.default_rng(4242 + r).random(COUNT_D, dtype=np.float32)
    x *= 2
    x -= 1
    return x


def _input_e_i64(r):
    return np.frombuffer(np.random.default_rng(5151 + r).bytes(COUNT_E_I64 * 8), dtype=np.int64)


def _input_e_f8(r):
    a = np.random.default_rng(6161 + r).integers(0, 256, COUNT_E_F8, dtype=np.uint8)
    a[(a & 0x7F) == 0x7F] &= 0xF7   # finite e4m3fn codes
    return a


def _digest(a):
    return hashlib.sha256(memoryview(np.ascontiguousarray(a)).cast("B")).hexdigest()


def _digest_e4m3(a):
    """Digest with every NaN code made 0x7F: NaN is compared as NaN, not by
    sign (the repo's parity convention, tests/test_reduce_gpu.py assert_same —
    the GPU's fp32 add returns a NaN whose sign need not be the x86 one's)."""
    return _digest(_canon_e4m3(a))


def _canon_e4m3(a):
    a = np.array(a, dtype=np.uint8, copy=True)
    a[(a & 0x7F) == 0x7F] = 0x7F
    return a


CHUNK_BYTES = 1 << 20


def _chunk_digests(a):
    """Short digests of every 1 MiB of an output: a wrong output then says WHERE
    it is wrong (mp_diag maps the chunks to the Simple schedule's cells)."""
    b = memoryview(np.ascontiguousarray(a)).cast("B")
    return [hashlib.sha256(b[o:o + CHUNK_BYTES]).hexdigest()[:16] for o in range(0, len(b), CHUNK_BYTES)]


def _describe_chunks(key, r, got, want, settings, algo):
    """Which 1 MiB chunks differ, as element ranges and (block, round, workgroup) cells."""
    from tests import mp_diag
    eb = {"d_allreduce": 4, "d_reduce_scatter": 4, "e_i64_max": 8, "e_f8_sum": 1}[key]
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    if len(got) != len(want):
        return f"{key} rank {r}: {len(got)} chunks vs {len(want)} expected"
    msg = f"{key} rank {r}: {len(bad)} of {len(want)} 1 MiB chunks differ, first {bad[:6]}"
    if settings and algo == "direct" and bad:
        kind, count = {"d_allreduce": ("ar", COUNT_D), "d_reduce_scatter": ("rs", RC_D),
                       "e_i64_max": ("ar", COUNT_E_I64), "e_f8_sum": ("ar", COUNT_E_F8)}[key]
        g = mp_diag.simple_geometry(kind, count, eb, N_RANKS, settings.get("simpleGrid", 32),
                                    settings.get("sliceBytes", 64 << 10))
        base = r * count if kind == "rs" else 0
        per = CHUNK_BYTES // eb
        idx = np.concatenate([np.arange(i * per, (i + 1) * per, max(per // 64, 1)) for i in bad[:64]])
        cells = np.unique(g.locate(idx + base)[:, :3], axis=0)
        msg += (f"; geometry block {g.block_elts} grid {g.grid} slice {g.slice_elts} rounds {g.n_rounds}; "
                f"{len(cells)} (block, round, workgroup) cells touched, e.g. {cells[:6].tolist()}")
    return msg


def _child_de(uid_bytes, rank, n, q):
    try:
        import torch
        from tests.conftest import load_package
        nbx = load_package()
        nbx.load_library()
        torch.cuda.set_device(0)
        comm = nbx.Communicator.init_rank(n, nbx.ncclUniqueId.from_buffer_copy(uid_bytes), rank)
        st = torch.cuda.current_stream().cuda_stream
        from tests import mp_diag
        res = {"settings": mp_diag.comm_settings(nbx, comm)}

        def timed(fn):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e3

        x = torch.from_numpy(_input_d(rank)).cuda()
        y = torch.empty_like(x)
        res["d_allreduce_ms"] = timed(lambda: comm.all_reduce(x.data_ptr(), y.data_ptr(), COUNT_D, F32, 0, st))
        yh = y.cpu().numpy()
        res["d_allreduce"], res["d_allreduce_chunks"] = _digest(yh), _chunk_digests(yh)
        del yh
        print(f"rank {rank}: config D AllReduce done ({res['d_allreduce_ms']:.1f} ms)", flush=True)
        z = torch.empty(RC_D, dtype=torch.float32, device="cuda")
        res["d_reduce_scatter_ms"] = timed(lambda: comm.reduce_scatter(x.data_ptr(), z.data_ptr(), RC_D, F32, 0, st))
        zh = z.cpu().numpy()
        res["d_reduce_scatter"], res["d_reduce_scatter_chunks"] = _digest(zh), _chunk_digests(zh)
        del x, y, z
        a = torch.from_numpy(_input_e_i64(rank).copy()).cuda()
        b = torch.empty_like(a)
        res["e_i64_max_ms"] = timed(lambda: comm.all_reduce(a.data_ptr(), b.data_ptr(), COUNT_E_I64, I64, 2, st))
        bh = b.cpu().numpy()
        res["e_i64_max"], res["e_i64_max_chunks"] = _digest(bh), _chunk_digests(bh)
        a = torch.from_numpy(_input_e_f8(rank)).cuda()
        b = torch.empty_like(a)
        res["e_f8_sum_ms"] = timed(lambda: comm.all_reduce(a.data_ptr(), b.data_ptr(), COUNT_E_F8, E4M3, 0, st))
        bh = _canon_e4m3(b.cpu().numpy())
        res["e_f8_sum"], res["e_f8_sum_chunks"] = _digest(bh), _chunk_digests(bh)
        print(f"rank {rank}: config E done", flush=True)
        assert comm.async_error() == 0
        comm.destroy()
        q.put((rank, "ok", res))
    except Exception:
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def _blocks(count, eb, n):
    epp = 16 // eb
    per = -(-count // n)
    per = -(-per // epp) * epp
    return [(min(count, per * b), min(count, per * b + per)) for b in range(n)]


def _ring_fold(oracle, xs, dtype, devop, arg, blocks, n):
    """Every block c folded in ring order c+1, ..., c (the direct schedule and
    NCCL's ring reduce-scatter accumulate block c in this order)."""
    out = np.empty(xs[0].size, dtype=xs[0].dtype)
    for c, (lo, hi) in enumerate(blocks):
        if hi > lo:
            order = [(c + 1 + k) % n for k in range(n)]
            oracle.reduce_multi([xs[j][lo:hi] for j in order], dtype, devop, arg, n_pre_op_srcs=n,
                                threads=16, out=[out[lo:hi]])
    return out


def _expected_de(oracle):
    n = N_RANKS
    exp = {}
    xs = [_input_d(r) for r in range(n)]
    _say("oracle: config D inputs regenerated")
    full = _ring_fold(oracle, xs, F32, 0, 0, _blocks(COUNT_D, 4, n), n)
    exp["d_allreduce"] = [(_digest(full), _chunk_digests(full))] * n
    rs = _ring_fold(oracle, xs, F32, 0, 0, [(c * RC_D, (c + 1) * RC_D) for c in range(n)], n)
    exp["d_reduce_scatter"] = [(_digest(rs[r * RC_D:(r + 1) * RC_D]), _chunk_digests(rs[r * RC_D:(r + 1) * RC_D]))
                               for r in range(n)]
    del xs, full, rs
    devop, arg = oracle.host_to_dev_redop(2, I64, n)   # ncclMax
    xs = [_input_e_i64(r) for r in range(n)]
    e = _ring_fold(oracle, xs, I64, devop, arg, _blocks(COUNT_E_I64, 8, n), n)
    exp["e_i64_max"] = [(_digest(e), _chunk_digests(e))] * n
    xs = [_input_e_f8(r) for r in range(n)]
    e = _canon_e4m3(_ring_fold(oracle, xs, E4M3, 0, 0, _blocks(COUNT_E_F8, 1, n), n))
    exp["e_f8_sum"] = [(_digest(e), _chunk_digests(e))] * n
    _say("oracle: configs D and E expected digests ready")
    return exp


@pytest.mark.parametrize("algo", ["direct", "ring"])
def test_configs_d_e_8_ranks_full_size(nbx, oracle, monkeypatch, algo):
    """Config D (8 x 1 GiB fp32 AllReduce + ReduceScatter) and config E (8-rank
    AllReduce: int64 max, fp8 e4m3 sum, 128 MiB) at full size, every rank's
    whole output bit-exact against the oracle."""
    monkeypatch.setenv("NBX_BOOTSTRAP_TIMEOUT", "300")
    monkeypatch.setenv("NBX_TIMEOUT_SEC", "240")
    monkeypatch.setenv("NCCL_ALGO", "Ring" if algo == "ring" else "")
    monkeypatch.setenv("NBX_SIMPLE_MAX_GRID", "32")    # 8 ranks' Simple grids co-resident on one GPU
    monkeypatch.setenv("NBX_LL128_MAX_GRID", "16")
    n = N_RANKS
    uid = nbx.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_child_de, args=(bytes(uid), r, n, q), daemon=True) for r in range(n)]
    for p in procs:
        p.start()
    res = {}
    try:
        exp = _expected_de(oracle)   # while the ranks run
        deadline = time.monotonic() + 600
        while len(res) < n:
            try:
                rank, status, payload = q.get(timeout=30)
            except Exception:
                assert time.monotonic() < deadline, f"ranks {sorted(set(range(n)) - set(res))} did not report"
                _say(f"waiting for ranks {sorted(set(range(n)) - set(res))}")
                continue
            assert status == "ok", f"rank {rank}:\n{payload}"
            res[rank] = payload
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
    wrong = []
    for key, digests in exp.items():
        for r in range(n):
            if res[r][key] != digests[r][0]:
                wrong.append(_describe_chunks(key, r, res[r][key + "_chunks"], digests[r][1], res[r].get("settings"),
                                              algo))
    if wrong:
        from tests import mp_diag
        head = f"configs D/E ({algo}): {len(wrong)} wrong output(s)"
        tail = mp_diag.emit_summary([head] + [w.split(";")[0] for w in wrong[:8]])
        raise AssertionError(head + ":\n" + "\n".join(wrong[:8]) + "\n" + tail)
    times = {k: round(max(res[r][k] for r in range(n)), 2) for k in res[0] if isinstance(k, str) and k.endswith("_ms")}
    print(f"configs D/E ({algo}, 8 ranks sharing one GPU), max ms over ranks: {times}", file=sys.stderr)
