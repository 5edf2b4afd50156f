"""bench.py's N > 1 leg budget on the CPU: two gloo ranks
run bench.main under torch.distributed.run with the GPU headline replaced by a
stub and every leg hanging — the multi-process collective child after one
partial result, the clique child, and the RCCL leg inside the bench process —
at the legs' DEFAULT timeouts (400 s each). The run must end inside the leg
budget (+ the watchdog's grace), exit non-zero (rank 0's status
bench.EXIT_LEG_CUT_OFF: a leg was cut off), and leave the headline value on
stdout twice: once before the legs, and last with `collective.ok` false and
the reason, carrying what the collective child reported before it hung."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

HANG_COLL = r'''
import json, os, sys, time
rank = int(os.environ["RANK"])
for line in sys.stdin:
    p = line.split()
    if p and p[0] == "ID":
        print("ID aa bb cc dd ee ff", flush=True)
    elif p and p[0] == "RUN":
        print("PARTIAL " + json.dumps({"rank": rank, "ok": True, "errors": [], "allreduce_direct_ms": 10.0 + rank,
                                       "stage": "config D timed"}), flush=True)
        if os.environ.get("STUB_MODE") == "hang" and os.environ.get("NBX_BENCH_COLLECTIVE_STUB_OK") != "1":
            time.sleep(600)
        print("RESULT " + json.dumps({"rank": rank, "ok": True, "errors": [], "allreduce_direct_ms": 10.0 + rank,
                                      "transport_allreduce_ms": 6.0, "reduce_scatter_ms": 5.0,
                                      "link_push_ms": 4.0 + rank, "link_pull_ms": 2.0, "link_bytes_per_peer": 1 << 28,
                                      "simple_knobs_ms": {"slice256K": 9.0 + rank, "grid64": 12.0, "slots4": 10.0},
                                      "curve_allreduce_ms": [1.0 + rank, 3.0],
                                      "ipc_repairs": {"direct": rank, "ring": 0},
                                      "ll128_forced_checked_calls": 2000, "ll128_forced_mismatched_calls": 0,
                                      "mixed_seq_checked_calls": 120 + rank, "mixed_seq_mismatches": rank}),
              flush=True)
        break
'''

HANG_CLIQUE = r'''
import json, os, sys, time
for line in sys.stdin:
    if line.startswith("RUN"):
        if os.environ.get("STUB_MODE") == "hang":
            time.sleep(600)
        print("RESULT " + json.dumps({"ok": True, "errors": [], "allreduce_ms": 8.0, "fold_allreduce_ms": 9.0}),
              flush=True)
        break
'''

DRIVER = r'''
import os, sys, time
sys.path.insert(0, os.environ["BENCH_ROOT"])
import bench
bench.COLLECTIVE_SCRIPT = os.environ["STUB_COLL"]
bench.CLIQUE_SCRIPT = os.environ["STUB_CLIQUE"]

def fake_headline(args, world, rank, local):   # the GPU timed region, stubbed
    m = bench.max_over_ranks(1.0 + rank, world)
    return {"metric": bench.METRIC, "value": 123.0, "n_gpus": world, "ms_per_step": m,
            "roofline": {"frac": 0.79}, "cpu_baseline": None, "collective": None}

bench.headline = fake_headline
if os.environ.get("STUB_MODE") == "hang":
    def hanging_rccl(world):
        time.sleep(3600)
    bench.rccl_leg = hanging_rccl
sys.exit(bench.main(["--gpus", "2", "--steps", "1", "--warmup", "0"]))
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp_path, mode, budget, leg_min, grace, **extra):
    for name, text in (("stub_coll.py", HANG_COLL), ("stub_clique.py", HANG_CLIQUE), ("driver.py", DRIVER)):
        (tmp_path / name).write_text(text)
    env = dict(os.environ, BENCH_ROOT=ROOT, STUB_COLL=str(tmp_path / "stub_coll.py"),
               STUB_CLIQUE=str(tmp_path / "stub_clique.py"), STUB_MODE=mode, NBX_BENCH_BACKEND="gloo",
               NBX_BENCH_LEG_BUDGET_S=str(budget), NBX_BENCH_LEG_MIN_S=str(leg_min),
               NBX_BENCH_WATCHDOG_GRACE_S=str(grace), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", **extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(tmp_path / "driver.py")]
    t0 = time.monotonic()
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    el = time.monotonic() - t0
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    return p, el, lines


def test_leg_timeout_is_capped_by_the_budget():
    assert bench.leg_timeout(400.0, 100.0, reserve=30.0) == 70.0
    assert bench.leg_timeout(400.0, 10.0, reserve=30.0) == 0.0
    assert bench.leg_timeout(60.0, 500.0) == 60.0
    # the default budget, with the watchdog's grace, keeps an 8-rank run far inside a 600 s driver limit
    assert bench.LEG_BUDGET_S + bench.WATCHDOG_GRACE_S <= 300
    b = bench.LegBudget(50.0, clock=iter([0.0, 20.0, 80.0]).__next__)
    assert b.left() == 30.0 and b.left() == 0.0


def test_skipped_leg_names_the_budget():
    s = bench.skipped_leg(3.0, "the clique leg")
    assert s["ok"] is False and "the clique leg skipped" in s["skipped"] and "NBX_BENCH_LEG_BUDGET_S" in s["skipped"]


def test_every_leg_hangs_the_run_ends_inside_the_budget(tmp_path):
    budget, leg_min, grace = 12.0, 3.0, 3.0
    p, el, lines = _run(tmp_path, "hang", budget, leg_min, grace)
    # the run says a leg was cut off: rank 0 exits EXIT_LEG_CUT_OFF, torchrun fails the job
    assert p.returncode != 0, p.stderr[-3000:]
    assert f"exitcode  : {bench.EXIT_LEG_CUT_OFF}" in p.stderr or f"exitcode: {bench.EXIT_LEG_CUT_OFF}" in p.stderr \
        or "ChildFailedError" in p.stderr, p.stderr[-3000:]
    # bounded by the budget + grace (+ process start-up and torch import), far below the legs' 400 s defaults
    assert el < budget + grace + 60, el
    assert len(lines) == 2, p.stdout
    first, last = lines
    assert first["value"] == 123.0 and first["collective"]["status"].startswith("pending")
    assert last["value"] == 123.0
    coll = last["collective"]
    assert coll["ok"] is False
    reasons = " ".join(coll.get("errors", []))
    # the collective child's partial result is kept (max over ranks) and its timeout named
    assert coll["allreduce_direct"]["ms"] == 11.0, coll
    assert "no result from the collective leg within" in reasons, reasons
    assert coll["clique"]["ok"] is False and coll["clique"]["incomplete"] is True
    # whatever was left for the RCCL leg: skipped with the reason, or ended by the watchdog
    assert (coll["rccl"] or {}).get("skipped") or "watchdog" in reasons, coll
    assert coll.get("leg_budget", {}).get("used_s", 0) <= budget + 1 or "watchdog" in reasons


def test_hang_inside_the_bench_process_ends_by_the_watchdog(tmp_path):
    """The RCCL leg runs in the bench process itself (no child to time out):
    the watchdog prints the final line and ends every rank at budget + grace."""
    budget, leg_min, grace = 10.0, 3.0, 3.0
    p, el, lines = _run(tmp_path, "hang", budget, leg_min, grace, NBX_BENCH_COLLECTIVE_STUB_OK="1",
                        NBX_BENCH_CLIQUE="0")
    assert p.returncode != 0, p.stderr[-3000:]   # the watchdog exits EXIT_LEG_CUT_OFF
    assert el < budget + grace + 60, el
    assert len(lines) == 2, p.stdout
    last = lines[-1]
    assert last["value"] == 123.0
    coll = last["collective"]
    assert coll["ok"] is False
    reasons = " ".join(coll.get("errors", []))
    assert "watchdog" in reasons and "RCCL" in reasons, reasons
    assert coll["allreduce_direct"]["ms"] == 11.0   # the legs' results before the hang are kept


def test_legs_finish_normally_inside_the_budget(tmp_path):
    p, el, lines = _run(tmp_path, "ok", 60.0, 3.0, 3.0)
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 2, p.stdout
    coll = lines[-1]["collective"]
    assert coll["ok"] is True, coll
    assert coll["clique"]["ok"] is True and coll["clique"]["fold_allreduce"]["hbm_GBs_per_rank"] > 0
    assert coll["rccl"] is None            # gloo: no RCCL leg
    assert coll["ipc_repairs"] == {"direct": 1, "ring": 0}
    assert coll["ll128_forced"]["checked_calls"] == 4000 and coll["ll128_forced"]["mismatched_calls"] == 0
    assert coll["mixed_seq"]["checked_calls"] == 241 and coll["mixed_seq"]["mismatches_per_rank"] == [0, 1]
    tr = coll["transport_allreduce"]
    S = bench.COUNT_D * 4
    assert tr["ms"] == 6.0
    n, M = 2, S
    model = 4 * (n - 1) * M // n + M // n + M
    assert tr["hbm_model_bytes_per_rank"] == model
    assert abs(tr["hbm_GBs_per_rank"] - round(model / 6e-3 / 1e9, 1)) < 1e-9
    ard = coll["allreduce_direct"]
    assert ard["hbm_model_bytes_per_rank"] == 2 * (M + 2 * (n - 1) * M // n)
    r = ard["hbm_over_model_applied"]
    assert abs(ard["hbm_GBs_per_rank"] - round(ard["hbm_model_bytes_per_rank"] * r / 11e-3 / 1e9, 1)) < 1e-9
    assert coll["leg_budget"]["budget_s"] == 60.0
    # the fabric: per-link rates from the slowest rank's probe, floors per entry
    fab = coll["fabric"]
    push, pull = (1 << 28) / 5e-3 / 1e9, (1 << 28) / 2e-3 / 1e9
    assert abs(fab["push_GBs_per_link"] - round(push, 2)) < 1e-9 and abs(fab["pull_GBs_per_link"] - round(pull, 2)) < 1e-9
    assert "fabric_rates" not in coll
    floor = 2 * M // n / (push * 1e9) * 1e3
    assert ard["fabric_link_bytes"] == 2 * M // n and abs(ard["fabric_floor_ms"] - round(floor, 4)) < 1e-9
    assert abs(ard["fabric_frac"] - round(floor / 11.0, 3)) < 1e-9
    rs = coll["reduce_scatter"]
    assert rs["fabric_link_bytes"] == M // n
    assert coll["simple_knobs"] == {"slice256K": 10.0, "grid64": 12.0, "slots4": 10.0, "default": 11.0}
    cu = coll["allreduce_curve"]
    assert cu["bytes"] == [64 << 20, 256 << 20] and cu["ms"] == [2.0, 3.0]
    assert abs(cu["busbw_GBs"][1] - round((256 << 20) / 3e-3 / 1e9, 2)) < 1e-9   # n = 2: busbw = algbw
    fa = coll["clique"]["fold_allreduce"]
    assert abs(fa["fabric_floor_ms"] - round(max(M // n / (pull * 1e9), M // n / (push * 1e9)) * 1e3, 4)) < 1e-9


def test_exit_status_contract():
    """0 for a complete run; EXIT_LEG_CUT_OFF when any leg ended without its result."""
    assert bench.EXIT_LEG_CUT_OFF not in (0, 1, 2)
    assert not bench.legs_cut_off(None) and not bench.legs_cut_off({"ok": True, "clique": {"ok": True}})
    assert bench.legs_cut_off({"ok": False, "incomplete": "watchdog"})
    assert bench.legs_cut_off({"ok": False, "clique": {"ok": False, "incomplete": True}})
    fired = []
    wd = bench.Watchdog(0.05, bench.Emitter(1), [], exit_fn=lambda: fired.append(1))
    wd.thread.join(5)
    assert fired == [1]


def test_vs_rccl_ratios_include_the_curve():
    coll = {"allreduce_direct": {"ms": 10.0}, "reduce_scatter": {"ms": 6.0}, "ll128_allreduce_1MiB_us": 20.0,
            "ll_allreduce_4KiB_us": 8.0, "allreduce_curve": {"bytes": [64 << 20, 256 << 20], "ms": [1.0, 3.0]},
            "protocol_sweep": {"bytes": bench.SWEEP_BYTES[:2], "LL": [5.0, 7.0], "Simple": [9.0, 6.0]}}
    rccl = {"ok": True, "allreduce": {"ms": 8.0}, "reduce_scatter": {"ms": 6.0}, "allreduce_1MiB_us": 25.0,
            "allreduce_4KiB_us": 10.0, "curve_allreduce_ms": [2.0, 3.0], "sweep_allreduce_us": [10.0, 6.0]}
    v = bench.vs_rccl(coll, rccl)
    assert v["allreduce_1GiB"] == 1.25 and v["reduce_scatter_1GiB"] == 1.0
    assert v["allreduce_curve"] == [0.5, 1.0]
    assert v["sweep_best_protocol"] == [0.5, 1.0]
    assert bench.vs_rccl(coll, {"ok": False}) is None


def test_fabric_fields_absent_without_probe_numbers():
    """A leg that never reached the link probe (or a rank without it) leaves
    the fabric fields out instead of reporting a rate from partial data."""
    out = {"allreduce_direct": {"ms": 10.0}}
    bench.add_fabric_rates(out, [{"link_push_ms": 2.0, "link_bytes_per_peer": 1 << 20}, {}], 2, 1 << 30)
    assert "fabric" not in out and "fabric_floor_ms" not in out["allreduce_direct"]
    out = {"allreduce_direct": {"ms": 10.0}, "allreduce_ring": None}
    bench.add_fabric_rates(out, [{"link_push_ms": 2.0, "link_bytes_per_peer": 1 << 20}] * 2, 2, 1 << 30)
    assert out["fabric"]["push_GBs_per_link"] == round((1 << 20) / 2e-3 / 1e9, 2) and out["fabric"]["pull_GBs_per_link"] is None
    assert out["allreduce_direct"]["fabric_link_bytes"] == (1 << 30) and out["allreduce_ring"] is None
