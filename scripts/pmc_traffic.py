#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of a bench run into profiles/.

Reads the kernel-trace stats CSV and the two separate PMC passes
(FETCH_SIZE, WRITE_SIZE — separate passes because TCC has 4 counter slots and
FETCH_SIZE takes 3; MI355X_MICROARCH.md §rocprofv3 PMC slots) and writes
profiles/pmc_latest.json with the HBM bytes per launch of the config-B kernel:

    hbm_bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024

FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads exactly half
of a wide coalesced streaming read (MI355X_MICROARCH.md §HBM), hence x2.
usage: pmc_traffic.py <run_dir> <out_dir> [source label, e.g. "round 3 run r3c"]
"""
import csv
import json
import os
import sys

KERNEL = "kReducePacks<nbx::FnSumF<nbx::TyF32>, 8,"
ALG = 9 * (64 << 20) * 4


def per_kernel(path, counter):
    vals = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    run, out = sys.argv[1], sys.argv[2]
    os.makedirs(out, exist_ok=True)
    fetch = per_kernel(os.path.join(run, "pmc_fetch", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(run, "pmc_write", "pmc_counter_collection.csv"), "WRITE_SIZE")
    stats = {}
    with open(os.path.join(run, "prof", "trace_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            if KERNEL in r["Name"]:
                stats = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                         "max_ns": float(r["MaxNs"])}
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    hbm = 2 * f_kib * 1024 + w_kib * 1024
    d = {
        "workload": "config_b_f32_sum_8x256MiB",
        "kernel": "nbx::kReducePacks<FnSumF<TyF32>, 8, 4>",
        "fetch_size_kib_per_launch": f_kib, "write_size_kib_per_launch": w_kib,
        "launches_measured": {"fetch": len(fetch), "write": len(write)},
        "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half of wide streaming reads)",
        "hbm_bytes_per_launch": int(hbm),
        "alg_bytes_per_launch": ALG,
        "traffic_over_alg": round(hbm / ALG, 4),
        "kernel_trace": stats,
        "kernel_trace_GBps": round(ALG / (stats["avg_ns"] * 1e-9) / 1e9, 1) if stats else None,
        "source": sys.argv[3] if len(sys.argv) > 3 else run,
    }
    with open(os.path.join(out, "pmc_latest.json"), "w") as f:
        json.dump(d, f, indent=2)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
