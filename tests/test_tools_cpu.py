"""CPU tests of the measurement tooling: the config-C profiler cuts a rocprofv3
kernel trace and PMC passes into cases at its marker dispatches, and the
per-case traffic it reports is (2 x FETCH_SIZE + WRITE_SIZE) KiB per call."""
import csv
import json
import os
import subprocess
import sys

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
