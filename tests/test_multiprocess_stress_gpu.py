"""Randomized multi-process stress (scripts/mp_stress.py) as a GPU test: every
rank draws the same random plan of AllReduce / ReduceScatter / Reduce calls
(datatypes, ops, sizes across LL / LL128 / Simple, two unordered streams per
rank, group boundaries with LL group launches), issues it without host
synchronisation and checks every output exactly. A short run here; the
evidence run is profiles/r3/mp_stress_r3l.jsonl (2 / 3 / 4 ranks x 30 plans)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n,seed", [(2, 11), (3, 12)])
def test_multiprocess_random_plans_exact(n, seed):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "mp_stress.py"), str(n), "6", str(seed)],
                         capture_output=True, text=True, timeout=220, cwd=ROOT)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert out.returncode == 0 and lines, out.stderr[-2000:]
    res = json.loads(lines[-1])
    assert len(res["ranks"]) == n, res
    for r, v in res["ranks"].items():
        assert "exception" not in v, v
        assert v["mismatches"] == 0 and v["async_ok"] and v["calls"] > 0, (r, v)
