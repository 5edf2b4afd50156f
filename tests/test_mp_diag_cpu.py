"""CPU tests of the GPU suite's diagnosis and ordering aids.

* tests/mp_diag.py turns a wrong multi-process result into a description
  (wrong-element count, first / last index, the Simple schedule's (block,
  round, workgroup) cells, what the wrong values equal). A synthetic mismatch
  is fed through it and the mapping checked against the host's cut
  (comm_mp_launch.cc mpLaunchSimple).
* conftest.py orders the GPU suite: the single-GPU parity core before the
  multi-process transport files, so `-x` cannot hide config B's oracle check.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from tests import mp_diag

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_block_range_matches_host_rule():
    # 1,000,003 int32 over 8 ranks: ceil(count / 8) rounded up to whole 16-B packs
    assert mp_diag.block_range(1000003, 4, 8, 0) == (0, 125004)
    assert mp_diag.block_range(1000003, 4, 8, 7) == (875028, 1000003)
    assert mp_diag.block_range(5, 4, 8, 3) == (5, 5)   # empty trailing blocks


def test_simple_geometry_gputest_r05_case():
    """GPUTEST_r05's red case: 8 ranks, int32, 1,000,003 elements, 32-workgroup
    Simple grid, 64 KiB staging slices -> one round of 32 slices of 3,908."""
    g = mp_diag.simple_geometry("ar", 1000003, 4, 8, 32, 64 << 10)
    assert (g.block_elts, g.grid, g.slice_elts, g.n_rounds) == (125004, 32, 3908, 1)
    # more workgroups than 4 KiB pieces: the grid shrinks; a small slice: many rounds
    g2 = mp_diag.simple_geometry("ar", 4096, 4, 2, 128, 64 << 10)
    assert (g2.block_elts, g2.grid, g2.n_rounds) == (2048, 2, 1)
    g3 = mp_diag.simple_geometry("rs", 100000, 4, 4, 2, 4096)
    assert (g3.block_elts, g3.grid, g3.slice_elts, g3.n_rounds) == (100000, 2, 1024, 49)


def test_describe_synthetic_mismatch_maps_cells_and_explanations():
    g = mp_diag.simple_geometry("ar", 1000003, 4, 8, 32, 64 << 10)
    rng = np.random.default_rng(1)
    srcs = [rng.integers(-2**31, 2**31 - 1, 1000003, dtype=np.int32) for _ in range(8)]
    exp = np.maximum.reduce(srcs)
    got = exp.copy()
    # block 3, workgroup 17: 40 elements lost rank 5's source; block 6, workgroup 2: 8 zeros
    lo = 3 * 125004 + 17 * 3908 + 100
    without5 = np.maximum.reduce([s for j, s in enumerate(srcs) if j != 5])
    idx = np.arange(lo, lo + 40)
    got[idx] = without5[idx]
    changed = idx[without5[idx] != exp[idx]]
    z0 = 6 * 125004 + 2 * 3908
    got[z0:z0 + 8] = 0
    d = mp_diag.describe_mismatch(got, exp, g, 0, {"without_rank5": without5, "raw_input_rank0": srcs[0]})
    assert d["n_wrong"] == changed.size + 8
    assert d["first"] == int(changed[0]) and d["last"] == z0 + 7
    assert d["explained_by"]["zero"] == 8
    assert d["explained_by"]["without_rank5"] == changed.size
    cells = {(c["block"], c["round"], c["workgroup"]): c["wrong"] for c in d["cells"]}
    assert cells == {(3, 0, 17): changed.size, (6, 0, 2): 8}
    assert d["first_at"][:3] == [3, 0, 17] and d["last_at"] == [6, 0, 2, 7]
    assert d["blocks"] == {3: changed.size, 6: 8}
    # assert_same raises with the description, and passes on equal data
    with pytest.raises(AssertionError, match=r"block.*workgroup"):
        mp_diag.assert_same(got.view(np.uint8), exp, ("ar", 2, 2, 1000003, 0), g)
    mp_diag.assert_same(exp.copy().view(np.uint8), exp, "equal")


def test_compact_summary_survives_a_3000_char_tail(capsys):
    """The round-end driver keeps the last 3,000 characters of the suite's
    output: the compact summary is printed last (captured stderr follows the
    assertion text) and stays short even for six wrong outputs."""
    g = mp_diag.simple_geometry("ar", 1000003, 4, 8, 32, 64 << 10)
    rng = np.random.default_rng(2)
    exp = rng.integers(-2**31, 2**31 - 1, 1000003, dtype=np.int32)
    got = exp.copy()
    got[500000:503908] = 0
    d = mp_diag.describe_mismatch(got, exp, g, 0, {})
    d["proto"] = "Simple"
    line = mp_diag.compact_mismatch(d)
    assert line.startswith("Simple 3908/1000003 wrong [500000..503907] 1 runs = zero=3908 cells")
    assert len(line) <= 160
    with pytest.raises(AssertionError) as ei:
        mp_diag.assert_same(got.view(np.uint8), exp, ("ar", 2, 2, 1000003, 0), g)
    err = capsys.readouterr().err
    assert err.startswith("SUMMARY ('ar', 2, 2, 1000003, 0): ?") and "wrong [500000..503907]" in err
    assert str(ei.value).rstrip().endswith(err.strip())
    six = " | ".join(["('ar', 2, 2, 1000003, 0) r7: " + line] * 6)
    assert len(six) < 1200


def test_check_equal_keeps_array_equal_semantics(capsys):
    """check_equal passes exactly when np.array_equal does (values, not dtypes)
    and describes a failure with the compact summary last."""
    a = np.arange(1000, dtype=np.int64)
    mp_diag.check_equal(a.astype(np.int32), a, "same values")
    mp_diag.check_equal(np.float32([0.0]), np.float32([-0.0]), "signed zero equal as values")
    b = a.astype(np.int32).copy()
    b[10:13] = -1
    with pytest.raises(AssertionError) as ei:
        mp_diag.check_equal(b, a, ("w0", 1000))
    assert "3 of 1000 elements wrong; first 10 last 12" in str(ei.value)
    assert str(ei.value).splitlines()[-1] == "SUMMARY ('w0', 1000): ? 3/1000 wrong [10..12] 1 runs"
    assert capsys.readouterr().err.strip() == str(ei.value).splitlines()[-1]


def test_describe_reduce_scatter_base_offset():
    """ReduceScatter output of rank r starts at send-side element r * recvcount."""
    g = mp_diag.simple_geometry("rs", 5000, 4, 4, 8, 4096)
    exp = np.arange(5000, dtype=np.float32)
    got = exp.copy()
    got[1500] = -1
    d = mp_diag.describe_mismatch(got, exp, g, base=2 * 5000)
    assert d["n_wrong"] == 1
    # 20,000-byte blocks: 5 workgroups of 1,000-element slices; offset 1500 -> workgroup 1, element 500
    assert (g.grid, g.slice_elts) == (5, 1000)
    assert d["first_at"] == [2, 0, 1, 500]


def test_gpu_suite_runs_single_gpu_core_first():
    out = subprocess.run([sys.executable, "-m", "pytest", "--collect-only", "-q", "-m", "gpu", "tests"], cwd=ROOT,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    files = []
    names = []
    for line in out.stdout.splitlines():
        if "::" in line:
            f = os.path.basename(line.split("::")[0])
            names.append(line)
            if not files or files[-1] != f:
                files.append(f)
    assert len(files) == len(set(files)), files   # each file in one contiguous run
    core = ["test_reduce_gpu.py", "test_config_a.py", "test_nccl_api_gpu.py"]
    assert files[:3] == core, files
    transport = [f for f in files if "multiprocess" in f or "stress" in f or "clique" in f]
    assert transport and min(files.index(f) for f in transport) > files.index("test_nccl_api_gpu.py")
    # config B's full-size oracle check comes before any multi-process test
    b = next(i for i, n in enumerate(names) if "test_config_b_full_size_bit_exact" in n)
    mp_first = next(i for i, n in enumerate(names) if "multiprocess" in n or "8_ranks" in n)
    assert b < mp_first
    # config C (one GPU) before configs D / E (8 ranks)
    c = max(i for i, n in enumerate(names) if "test_config_c" in n)
    de = min(i for i, n in enumerate(names) if "test_configs_d_e" in n)
    assert c < de


def test_diagnose_collective_names_the_missing_source_and_cell(capsys):
    """GPUTEST_r05's case as a synthetic failure: 8 ranks, int32 max over
    1,000,003 elements (Simple direct at the shared-GPU grid of 32); rank 0's
    output has one workgroup's slice of block 6 folded without rank 3's source.
    The description names the protocol, the cell and the missing source."""
    from oracle import oracle
    oracle.build()
    n, count = 8, 1000003
    xs = oracle.random_inputs(2, 8, count, seed=77 + 2 + count)
    devop, arg = oracle.host_to_dev_redop(2, 2, n)
    settings = {"llMax": 64 << 10, "l128Max": 1 << 20, "sliceBytes": 64 << 10, "simpleGrid": 32}
    full = np.empty(count, dtype=np.int32)
    for b in range(n):
        lo, hi = mp_diag.block_range(count, 4, n, b)
        order = [(b + 1 + k) % n for k in range(n)]
        full[lo:hi] = oracle.reduce_multi([xs[j][lo:hi] for j in order], 2, devop, arg, n_pre_op_srcs=n)[0]
    lo = 6 * 125004 + 9 * 3908
    idx = np.arange(lo, lo + 3908)
    without3 = np.maximum.reduce([xs[j][idx] for j in range(n) if j != 3])
    got = full.copy()
    got[idx] = without3
    changed = int((without3 != full[idx]).sum())
    assert changed > 0
    d = mp_diag.diagnose_collective(oracle, "ar", 2, 2, count, n, 0, got.view(np.uint8), xs, settings)
    assert d["proto"] == "Simple" and d["n_wrong"] == changed
    assert d["explained_by"]["without_rank3"] == changed
    assert [(c["block"], c["round"], c["workgroup"]) for c in d["cells"]] == [(6, 0, 9)]
    with pytest.raises(AssertionError, match=r"without_rank3=.*\(block, round, workgroup\)") as ei:
        mp_diag.raise_collective_failures(oracle, [("case 36", "ar", 2, 2, count, 0, got.view(np.uint8), xs,
                                                    settings, 1)], n)
    # the compact form closes the message and goes to stderr (the end of a truncated log)
    summary = (f"SUMMARY 1 wrong output(s) at 8 ranks | case 36 r0: Simple {changed}/{count} wrong "
               f"[{int(idx[without3 != full[idx]][0])}..")
    assert str(ei.value).splitlines()[-1].startswith(summary)
    last = str(ei.value).splitlines()[-1]
    assert f" = without_rank3={changed}," in last and last.endswith(f" cells 1 top b6r0w9:{changed}")
    assert len(last) < 250
    assert capsys.readouterr().err.startswith(summary)
    # protocol choice as comm_mp_init.cc chooseProtoFor at these settings
    assert mp_diag.proto_of("ar", 1000, 4, 8, settings) == "LL"
    assert mp_diag.proto_of("ar", 50003, 4, 8, settings) == "LL128"
    assert mp_diag.proto_of("ar", 262144, 4, 8, settings) == "LL128x2"
    assert mp_diag.proto_of("ar", 300000, 4, 8, settings) == "Simple"
    assert mp_diag.proto_of("rs", 131072, 4, 8, settings) == "LL128"


def test_proto_of_matches_the_library():
    """mp_diag.proto_of restates comm_mp_init.cc chooseProtoFor: checked
    against the library's own (nbxDebugChooseProto) over sizes, kinds, ranks."""
    import ctypes
    from tests.conftest import load_package
    lib = load_package().load_library()
    lib.nbxDebugChooseProto.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                        ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
    names = {0: "LL", 1: "LL128", 2: "Simple", 3: "LL128x2"}
    settings = {"llMax": 64 << 10, "l128Max": 1 << 20}
    for n in (2, 3, 5, 8, 9):
        for kind in ("ar", "rs", "red"):
            for eb in (1, 2, 4, 8):
                for count in (1, 17, 4097, 16384, 50003, 65537, 200001, 262144, 300001, 1000003):
                    lo, hi = mp_diag.block_range(count, eb, n, 0)
                    lib_p = lib.nbxDebugChooseProto(7, int(kind != "rs"), count * eb, (hi - lo) * eb, n, 64 << 10,
                                                    1 << 20, 256 << 10)
                    assert mp_diag.proto_of(kind, count, eb, n, settings) == names[lib_p], (n, kind, eb, count)


def test_configs_d_e_chunk_description():
    """The 8-rank config D / E test compares 1 MiB chunk digests on a mismatch
    and maps the differing chunks to the Simple schedule's cells."""
    from tests import test_configs_gpu as t
    a = np.arange(4 * t.CHUNK_BYTES // 4, dtype=np.float32)
    want = t._chunk_digests(a)
    b = a.copy()
    b[t.CHUNK_BYTES // 4 * 2 + 5] = -1   # chunk 2
    got = t._chunk_digests(b)
    msg = t._describe_chunks("d_allreduce", 0, got, want, {"simpleGrid": 32, "sliceBytes": 64 << 10}, "direct")
    assert "1 of 4 1 MiB chunks differ, first [2]" in msg and "(block, round, workgroup) cells" in msg


def test_mp_stress_describes_a_wrong_output():
    """scripts/mp_stress.py records what a wrong output looks like (bf16 too)."""
    import importlib.util
    import torch
    spec = importlib.util.spec_from_file_location("mp_stress", os.path.join(ROOT, "scripts", "mp_stress.py"))
    ms = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ms)
    ref = torch.arange(1, 1000001, dtype=torch.float32).to(torch.bfloat16)
    y = ref.clone()
    y[1000:1010] = 0
    c = {"kind": "allreduce", "count": 1000000}
    out = ms._describe(torch, c, y, ref, 0, 4, {"llMax": 64 << 10, "l128Max": 1 << 20, "simpleGrid": 64,
                                                 "sliceBytes": 64 << 10})
    assert out["what"].startswith("Simple: 10 of 1000000 elements wrong") and "zero=10" in out["what"]
