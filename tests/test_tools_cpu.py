"""CPU tests of the measurement tooling: the config-C profiler cuts a rocprofv3
kernel trace and PMC passes into cases at its marker dispatches, and the
per-case traffic it reports is (2 x FETCH_SIZE + WRITE_SIZE) KiB per call."""
import csv
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MARKER = "void nbx::kReducePacks<nbx::FnSumF<nbx::TyF32>, 3, 1>(nbx::KArgs)"
K16 = "void nbx::kReducePacks<nbx::FnSumF<nbx::TyF16>, 2, 1>(nbx::KArgs)"
K16B = "void nbx::kReduceBatch<nbx::FnSumF<nbx::TyF16>, 2>(nbx::BatchArgs)"


def _write_csv(path, header, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_config_c_summarize_cuts_cases_at_markers(tmp_path):
    # warmup dispatches before the first marker and a foreign kernel between
    # cases are ignored; case a: 2 calls x 1 dispatch, case b: 2 calls x 2 dispatches
    trace = [("at::native::fill", 0, 1), (K16, 1, 2), (MARKER, 10, 11), (K16, 12, 22), (K16, 23, 33),
             (MARKER, 34, 35), ("at::native::rand", 36, 37), (MARKER, 40, 41), (K16, 42, 52), (K16B, 53, 63),
             (K16, 64, 74), (K16B, 75, 85), (MARKER, 90, 91)]
    _write_csv(tmp_path / "trace.csv", ["Kernel_Name", "Start_Timestamp", "End_Timestamp"], trace)
    pmc = []
    for i, (name, _, _) in enumerate(trace):
        pmc.append([i + 1, name, "FETCH_SIZE", 1.0])
        pmc.append([i + 1, name, "WRITE_SIZE", 2.0])
    _write_csv(tmp_path / "pmc.csv", ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"], pmc)
    with open(tmp_path / "cases.jsonl", "w") as f:
        for c in ("a", "b"):
            f.write(json.dumps({"dtype": "fp16", "nsrc": 2, "case": c, "calls": 2, "alg_bytes_per_call": 4096}) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "config_c_profile.py"), "--summarize",
                          str(tmp_path / "cases.jsonl"), str(tmp_path / "trace.csv"), str(tmp_path / "pmc.csv")],
                         capture_output=True, text=True, check=True).stdout
    rows = [json.loads(l) for l in out.splitlines()]
    assert [r["case"] for r in rows] == ["a", "b"]
    a, b = rows
    assert a["rocprof_dispatches_per_call"] == 1.0 and b["rocprof_dispatches_per_call"] == 2.0
    assert a["rocprof_ms_per_call"] == 10 / 1e6 and b["rocprof_ms_per_call"] == 20 / 1e6   # ns -> ms
    # (2 x 1 + 2) KiB per dispatch
    assert a["hbm_bytes_per_call"] == 4096 and b["hbm_bytes_per_call"] == 8192
    assert a["traffic_over_alg"] == 1.0 and b["traffic_over_alg"] == 2.0
    assert b["kernels"] == sorted(["kReduceBatch<nbx::FnSumF<nbx::TyF16>, 2>", "kReducePacks<nbx::FnSumF<nbx::TyF16>, 2, 1>"])


def test_config_c_summarize_rejects_case_count_mismatch(tmp_path):
    _write_csv(tmp_path / "trace.csv", ["Kernel_Name", "Start_Timestamp", "End_Timestamp"],
               [(MARKER, 0, 1), (K16, 2, 3), (MARKER, 4, 5)])
    with open(tmp_path / "cases.jsonl", "w") as f:
        for c in ("a", "b"):
            f.write(json.dumps({"case": c, "calls": 1, "alg_bytes_per_call": 1}) + "\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "config_c_profile.py"), "--summarize",
                        str(tmp_path / "cases.jsonl"), str(tmp_path / "trace.csv")], capture_output=True, text=True)
    assert r.returncode == 1 and "1 trace segments for 2 cases" in r.stdout


# ---------------------------------------------------------------------------
# scripts/set_thresholds.py: protocol thresholds from a bench line's sweep


def _thr():
    import importlib.util
    spec = importlib.util.spec_from_file_location("set_thresholds", os.path.join(ROOT, "scripts", "set_thresholds.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_set_thresholds_on_the_r4_rehearsal():
    """The committed 2-rank shared-GPU line (r4aj): LL wins every swept size,
    so LL carries up to 1 MiB and LL128 nothing; the ring's 1 GiB beats the
    direct schedule by > 5 %; a shared-GPU run never enables LL128 across GPUs."""
    st = _thr()
    b = st.last_collective_line(os.path.join(ROOT, "profiles", "r4", "bench_n2_shared_r4aj.json"))
    b["shared_gpu"] = True
    r = st.thresholds(b)
    assert [row["chosen"] for row in r["rows"]] == ["LL"] * 4
    env = r["env"]
    assert env["NBX_LL_MAX_BYTES"] == 1 << 20 and env["NBX_LL128_MAX_BYTES"] == 0
    assert env["NCCL_ALGO"] == "Ring"              # 1.7984 ms direct vs 1.7064 ms ring
    assert env["NBX_CLIQUE_SIMPLE_MAX_BYTES"] == 32 << 20   # in-kernel 0.710 vs fold 0.733: inside the margin
    assert env["NBX_LL128_ACROSS_GPUS"] == ""
    assert "NBX_LL128_ONESHOT_MAX" not in env      # n = 2: no two-shot


def test_set_thresholds_synthetic_8_ranks_with_hysteresis():
    """A synthetic 8-GPU sweep: LL -> LL128 (one-shot, then two-shot) ->
    Simple; a 3 % win does not switch (hysteresis), a 20 % win does; a clean
    forced-LL128 stress on distinct GPUs enables LL128 across GPUs."""
    st = _thr()
    sizes = [4 << 10, 32 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20]
    sweep = {"bytes": sizes,
             "LL":            [9.0, 10.0, 30.0, 90.0, 300.0, 1200.0],
             "LL128":         [12.0, 9.8, 20.0, 28.0, 80.0, 300.0],    # 32 KiB: 2 % faster than LL -> stay
             "LL128_oneshot": [12.0, 9.8, 20.0, 40.0, 150.0, 600.0],   # one-shot up to 256 KiB
             "Simple":        [40.0, 42.0, 45.0, 50.0, 60.0, 90.0]}
    b = {"n_gpus": 8, "collective": {"n_ranks": 8, "protocol_sweep": sweep,
                                     "allreduce_direct": {"ms": 10.0}, "allreduce_ring": {"ms": 10.2},
                                     "clique": {"allreduce_ms": 8.0, "fold_allreduce_ms": 12.0},
                                     "ll128_forced": {"checked_calls": 16000, "mismatched_calls": 0}}}
    r = st.thresholds(b)
    assert [row["chosen"] for row in r["rows"]] == ["LL", "LL", "LL128", "LL128", "Simple", "Simple"]
    env = r["env"]
    assert env["NBX_LL_MAX_BYTES"] == 32 << 10
    assert env["NBX_LL128_MAX_BYTES"] == 1 << 20
    assert env["NBX_LL128_ONESHOT_MAX"] == 256 << 10
    assert env["NCCL_ALGO"] == ""                       # ring 2 % slower: direct stays
    assert env["NBX_CLIQUE_SIMPLE_MAX_BYTES"] == 1 << 40
    assert env["NBX_LL128_ACROSS_GPUS"] == "1"
    b["collective"]["ll128_forced"]["mismatched_calls"] = 1   # one torn line anywhere: keep it off
    assert st.thresholds(b)["env"]["NBX_LL128_ACROSS_GPUS"] == ""
    # Simple knobs: no sweep -> every knob unset; a 3 % win keeps the default; a 20 % win sets it
    assert env["NBX_SIMPLE_SLICE_BYTES"] == "" and env["NBX_SIMPLE_MAX_GRID"] == "" and env["NBX_SIMPLE_SLOTS"] == ""
    b["collective"]["simple_knobs"] = {"slice256K": 9.7, "grid64": 11.0, "slots4": 10.5, "default": 10.0}
    assert st.thresholds(b)["env"]["NBX_SIMPLE_SLICE_BYTES"] == ""
    b["collective"]["simple_knobs"]["grid64"] = 8.0
    e2 = st.thresholds(b)["env"]
    assert e2["NBX_SIMPLE_MAX_GRID"] == "64" and e2["NBX_SIMPLE_SLICE_BYTES"] == "" and e2["NBX_SIMPLE_SLOTS"] == ""


def test_set_thresholds_cli(tmp_path):
    import subprocess
    import sys
    p = tmp_path / "b.json"
    p.write_text("not json\n" + open(os.path.join(ROOT, "profiles", "r4", "bench_n2_shared_r4aj.json")).read())
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "set_thresholds.py"), str(p), "--shared-gpu"],
                         capture_output=True, text=True, check=True).stdout
    assert "export NBX_LL_MAX_BYTES=1048576" in out and "unset NBX_LL128_ACROSS_GPUS" in out


def test_set_thresholds_on_the_r5_rehearsal_with_knobs():
    """The committed N = 4 shared-GPU line with the Simple-knob sweep (r5z): the
    default knobs win there, so every knob stays unset; the line parses with
    every round-5 field present."""
    st = _thr()
    b = st.last_collective_line(os.path.join(ROOT, "profiles", "r5", "bench_n4_shared_r5z.json"))
    assert set(b["collective"]["simple_knobs"]) == {"slice256K", "grid64", "slots4", "default"}
    r = st.thresholds(b)
    env = r["env"]
    assert env["NBX_SIMPLE_SLICE_BYTES"] == "" and env["NBX_SIMPLE_MAX_GRID"] == "" and env["NBX_SIMPLE_SLOTS"] == ""
    assert env["NBX_LL128_ACROSS_GPUS"] == ""   # ranks shared one GPU


def test_collective_leg_mixed_cases_match_the_gpu_test_and_check_exactly():
    """scripts/collective_leg.py replays the GPU suite's LL_CASES on the node
    (VERDICT r5 item 4): the same list, and its torch restatement is exact for
    every case's leg op (on the CPU here: inputs, the expected result, and a
    wrong element detected)."""
    import importlib.util
    import torch
    from tests.test_multiprocess_gpu import LL_CASES
    spec = importlib.util.spec_from_file_location("collective_leg", os.path.join(ROOT, "scripts", "collective_leg.py"))
    leg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(leg)
    assert leg.MIXED_CASES == LL_CASES
    world = 3
    for i, (kind, dt, op0, count, shift) in enumerate(leg.MIXED_CASES):
        op = leg._mixed_op(op0)
        assert op in (0, 2, 3)
        total = min(count * world if kind == "rs" else count, 5000)
        ins = [leg._mixed_input(torch, dt, op, total, 100 * i + r, device="cpu") for r in range(world)]
        assert all(x.dtype == torch.uint8 and x.numel() == total * leg._EB[dt] for x in ins)
        want = leg._mixed_expected(torch, dt, op, ins)
        assert want.numel() == total * leg._EB[dt]
        # the restatement against a plain reference on a few elements
        ref = _plain_fold(np, dt, op, [x.numpy() for x in ins])
        assert np.array_equal(want.numpy(), ref), (i, dt, op)


def _plain_fold(np_, dt, op, ins):
    """numpy reference of the leg's op on raw bytes (floats through float64;
    fp8 through the oracle's decoders)."""
    from oracle import oracle as o
    st = {0: np_.int8, 1: np_.uint8, 2: np_.int32, 3: np_.uint32, 4: np_.int64, 5: np_.uint64, 6: np_.float16,
          7: np_.float32, 8: np_.float64}
    if dt in (10, 11):
        dec = o.e4m3_to_f32 if dt == 10 else o.e5m2_to_f32
        enc = o.f32_to_e4m3 if dt == 10 else o.f32_to_e5m2
        vals = [np_.array([dec(int(c)) for c in x], dtype=np_.float64) for x in ins]
        acc = sum(vals) if op == 0 else (np_.maximum.reduce(vals) if op == 2 else np_.minimum.reduce(vals))
        return np_.array([enc(float(v)) for v in acc], dtype=np_.uint8)
    if dt == 9:
        vals = [(x.view(np_.uint16).astype(np_.uint32) << 16).view(np_.float32).astype(np_.float64) for x in ins]
        acc = sum(vals) if op == 0 else (np_.maximum.reduce(vals) if op == 2 else np_.minimum.reduce(vals))
        return np_.array([o.f32_to_bf16(float(v)) for v in acc], dtype=np_.uint16).view(np_.uint8)
    vals = [x.view(st[dt]) for x in ins]
    if op == 0:
        acc = sum(v.astype(np_.float64) if dt in (6, 7, 8) else v.astype(np_.int64) for v in vals)
        return acc.astype(st[dt]).view(np_.uint8)
    f = np_.maximum if op == 2 else np_.minimum
    return f.reduce(vals).view(np_.uint8)


def test_clique_stress_refuses_more_streams_than_hardware_queues():
    """scripts/clique_stress.py: the rank counts of one process must fit the
    hardware queues (a shared queue deadlocks the in-kernel transport on the
    one-GPU rig, profiles/r6/clique_queues_r6x/); refused before HIP loads."""
    script = os.path.join(ROOT, "scripts", "clique_stress.py")
    env = {k: v for k, v in os.environ.items() if k != "NBX_STRESS_HW_QUEUES"}
    out = subprocess.run([sys.executable, script, "2,3,4,8", "1", "1"], capture_output=True, text=True,
                         timeout=60, env=env)
    assert out.returncode != 0 and "need 30 streams" in out.stderr and "24 hardware queues" in out.stderr
    out = subprocess.run([sys.executable, script, "8,8,8,8", "1", "1"], capture_output=True, text=True,
                         timeout=60, env=dict(env, NBX_STRESS_HW_QUEUES="40"))   # clamped to 32
    assert out.returncode != 0 and "need 36 streams" in out.stderr and "32 hardware queues" in out.stderr
    code = ("import sys; sys.path.insert(0, 'scripts'); import clique_stress as c; "
            "print([c.streams_needed(ns) for ns in ([2, 3], [4], [2, 3, 4], [8, 8], [8, 8, 8])])")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, cwd=ROOT, env=env)
    assert out.stdout.strip() == "[12, 9, 21, 18, 27]", out.stderr
