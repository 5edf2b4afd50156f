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


@pytest.mark.parametrize("seed,dyn_min_tiles", [(11, 0), (12, 1)])
def test_scheduling_stress(torch_gpu, seed, dyn_min_tiles):
    """dyn_min_tiles 0: the library's default tile policy; 1: every big-tile
    launch dynamic (the stress sizes are below the default threshold)."""
    rc, res = _stress_module().main(["--ops", "400", "--seed", str(seed), "--dyn-min-tiles", str(dyn_min_tiles)])
    assert rc == 0 and res["mismatches"] == 0, res
