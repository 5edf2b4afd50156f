"""The in-process clique's in-kernel LL / LL128 transport (cliqueInitTransport,
comm_clique.cc) as a GPU test: scripts/clique_stress.py forces it on for ranks
sharing the one GPU of the test box (NBX_CLIQUE_LL=1, each rank on its own
streams and hardware queues, both set in that fresh process before HIP loads),
runs random plans of AllReduce / ReduceScatter / Reduce across LL, LL128 one-
and two-shot and the Simple-sized fold path, with groups, stream switches and
calls whose ranks share one stream (fold path), and checks every rank's output
exactly. On a node whose clique ranks sit on distinct GPUs the transport is on
by default."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("ranks,seed,simple", [("2,3", 21, "1"), ("4", 22, "1"), ("3", 23, "0")])
def test_clique_in_kernel_transport_random_plans_exact(ranks, seed, simple):
    """simple = 1 (default): Simple-sized calls run in-kernel too (the
    multi-process Simple kernels over the clique's staging); 0: they keep the
    event-ordered fold path."""
    env = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "NBX_CLIQUE_LL")}
    env["NBX_CLIQUE_SIMPLE"] = simple
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "clique_stress.py"), ranks, "5", str(seed)],
                         capture_output=True, text=True, timeout=220, cwd=ROOT, env=env)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert out.returncode == 0 and len(lines) == len(ranks.split(",")), out.stderr[-2000:]
    for ln in lines:
        res = json.loads(ln)
        assert res["in_kernel"], res          # the transport is active on every rank
        assert res["checked"] > 0 and res["mismatches"] == 0 and res["async_ok"], res
