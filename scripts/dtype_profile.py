#!/usr/bin/env python3
"""dtype_profile.py — one 8-source reduction case, launched `iters` times
back to back after 2 warm-ups, for rocprofv3 kernel-trace / PMC passes
(attribute fp8's lower roofline fraction). Inputs as
probe_dtypes.py (fp8: random finite codes; floats: uniform [0, 1)), one
output. Prints one JSON line: HIP-event device ms per launch, algorithmic
bytes per launch (9 x input bytes), TB/s.
usage: dtype_profile.py datatype redop eltbytes MiB_per_input iters [blocksPerCU variant]
  e.g. 10 0 1 128 10  (fp8 e4m3 sum, config E shape)
       7 0 4 128 10   (fp32 sum, same bytes)
  blocksPerCU / variant: nbxSetLaunchConfig (0 = default; variant 1 small
  tiles, 2 big tiles) for launch-shape A/B in separate processes.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    dt, redop, esz, mib, iters = (int(v) for v in sys.argv[1:6])
    bpc, variant = (int(sys.argv[6]), int(sys.argv[7])) if len(sys.argv) > 7 else (0, 0)
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    lib = nbx.load_library()
    if lib.nbxSetLaunchConfig(bpc, variant) != 0:
        raise SystemExit("bad launch config")
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    n = (mib << 20) // esz
    g = torch.Generator(device="cuda").manual_seed(5)
    srcs = []
    for _ in range(8):
        if dt in (10, 11):
            b = torch.randint(0, 256, (mib << 20,), dtype=torch.uint8, device="cuda", generator=g) & 0x77
        elif dt in (6, 9, 7):
            b = torch.rand(n, device="cuda", generator=g).to({6: torch.float16, 9: torch.bfloat16,
                                                                7: torch.float32}[dt]).view(torch.uint8)
        else:
            b = torch.randint(0, 256, (mib << 20,), dtype=torch.uint8, device="cuda", generator=g)
        srcs.append(b)
    out = torch.empty(mib << 20, dtype=torch.uint8, device="cuda")
    sp = [t.data_ptr() for t in srcs]
    op = nbx.host_to_dev_redop(redop, dt, 8)
    for _ in range(2):
        nbx.reduce_multi([out.data_ptr()], sp, n, dt, op, 0, False, st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(iters):
        nbx.reduce_multi([out.data_ptr()], sp, n, dt, op, 0, False, st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    alg = 9 * (mib << 20)
    print(json.dumps({"datatype": dt, "redop": redop, "MiB_per_input": mib, "n_srcs": 8, "launches": iters + 2,
                      "blocks_per_cu": bpc, "variant": variant,
                      "ms": round(ms, 5), "alg_bytes": alg, "TBps": round(alg / (ms * 1e-3) / 1e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
