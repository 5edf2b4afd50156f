"""bench.py host logic on the CPU: the libnbxccl-vs-RCCL ratio summary of the
N > 1 collective leg (time ratios, per-size best protocol) and its tolerance
of missing pieces."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_vs_rccl_ratios():
    coll = {"allreduce_direct": {"ms": 2.0}, "reduce_scatter": {"ms": 1.0}, "ll128_allreduce_1MiB_us": 30.0,
            "ll_allreduce_4KiB_us": 5.0,
            "protocol_sweep": {"bytes": [4096, 32768], "LL": [5.0, 6.0], "LL128": [7.0, 6.5], "LL128_oneshot": None,
                               "Simple": [20.0, 3.0]}}
    rccl = {"ok": True, "allreduce": {"ms": 4.0}, "reduce_scatter": {"ms": 2.0}, "allreduce_1MiB_us": 40.0,
            "allreduce_4KiB_us": 10.0, "sweep_allreduce_us": [10.0, 12.0, 1, 1, 1, 1]}
    v = bench.vs_rccl(coll, rccl)
    assert v["allreduce_1GiB"] == 0.5 and v["reduce_scatter_1GiB"] == 0.5
    assert v["allreduce_1MiB"] == 0.75 and v["allreduce_4KiB"] == 0.5
    assert v["sweep_best_protocol"] == [0.5, 0.25]   # per size: fastest protocol / RCCL


def test_vs_rccl_missing_pieces():
    assert bench.vs_rccl(None, {"ok": True}) is None
    assert bench.vs_rccl({"allreduce_direct": None}, {"ok": False}) is None
    v = bench.vs_rccl({"allreduce_direct": None, "reduce_scatter": None}, {"ok": True})
    assert v["allreduce_1GiB"] is None and "sweep_best_protocol" not in v


def test_simple_hbm_model():
    m = bench.simple_hbm_model(2, 1 << 30)
    assert m["algorithmic_bytes_per_rank"] == 2 << 30
    assert m["staging_model_bytes_per_rank"] == 4 << 30      # n = 2: twice the user-visible bytes
    assert m["xgmi_bytes_per_rank_each_way"] == 1 << 30
    m8 = bench.simple_hbm_model(8, 1 << 30)
    assert m8["staging_model_bytes_per_rank"] == 2 * ((1 << 30) + 2 * 7 * (1 << 30) // 8)
    if m8["measured_over_model"] is not None:                 # the committed PMC summary
        assert 0.95 < m8["measured_over_model"]["direct"] < 1.1
