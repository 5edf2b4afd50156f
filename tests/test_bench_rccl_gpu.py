"""bench.py's N > 1 RCCL code on the GPU: the
bench's process-group init with backend "nccl" (device_id given),
max_over_ranks through an RCCL all-reduce, rccl_leg's config-D shapes and
sweep, and vs_rccl over its output — at one rank, in a fresh child process
that joins the group before any other GPU call (RCCL refuses two ranks on one
GPU, so one rank is what a one-GPU box can run). The driver's multi-GPU bench
is then not the first execution of any of it."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CHILD = r"""
import json, os, sys
sys.path.insert(0, sys.argv[1])
import torch
import torch.distributed as dist
import bench
bench.init_process_group("nccl", 0, 1, 0)   # before any other GPU call of this process
torch.cuda.set_device(0)
assert dist.get_backend() == "nccl"
m = bench.max_over_ranks(3.25, 1)           # the all-reduce path, not the world == 1 shortcut
r = bench.rccl_leg(1)
coll = {"allreduce_direct": {"ms": 2.0}, "reduce_scatter": {"ms": 1.0}, "ll128_allreduce_1MiB_us": 30.0,
        "ll_allreduce_4KiB_us": 5.0,
        "protocol_sweep": {"bytes": list(bench.SWEEP_BYTES), "LL": [5.0] * 6, "LL128": [4.0] * 6,
                           "LL128_oneshot": None, "Simple": [3.0] * 6}}
v = bench.vs_rccl(coll, r)
dist.destroy_process_group()
print("RESULT " + json.dumps({"max": m, "rccl": r, "vs": v}), flush=True)
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_bench_rccl_leg_one_rank_nccl_backend():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-4000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, p.stdout[-2000:] + p.stderr[-2000:]
    res = json.loads(line[-1][len("RESULT "):])
    assert res["max"] == 3.25
    r = res["rccl"]
    assert r["ok"] is True, r
    for key in ("allreduce", "reduce_scatter", "allgather_transport"):
        assert r[key]["ms"] > 0 and r[key]["algbw_GBs"] > 0, (key, r[key])
        assert "busbw_GBs" in r[key]
    assert r["sweep_bytes"] == list(bench.SWEEP_BYTES)
    assert len(r["sweep_allreduce_us"]) == 6 and all(t > 0 for t in r["sweep_allreduce_us"])
    assert r["allreduce_1MiB_us"] > 0 and r["allreduce_4KiB_us"] > 0
    v = res["vs"]
    assert v is not None and v["allreduce_1GiB"] > 0 and v["reduce_scatter_1GiB"] > 0
    assert len(v["sweep_best_protocol"]) == 6 and all(x is not None and x > 0 for x in v["sweep_best_protocol"])
