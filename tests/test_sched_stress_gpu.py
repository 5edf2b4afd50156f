"""Randomized stress of the launch machinery (dynamic tile counters, work-list
table slots, graph-owned slots, kernel-argument fallbacks) across four streams
with graph captures — scripts/stress_sched.py at a test-sized count, in this
process, every output checked exactly (small-integer fp32 data)."""
import importlib.util
import os

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stress_module():
    spec = importlib.util.spec_from_file_location("stress_sched", os.path.join(ROOT, "scripts", "stress_sched.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("seed", [11, 12])
def test_scheduling_stress(torch_gpu, seed):
    rc, res = _stress_module().main(["--ops", "400", "--seed", str(seed)])
    assert rc == 0 and res["mismatches"] == 0, res
