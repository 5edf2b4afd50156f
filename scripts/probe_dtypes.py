#!/usr/bin/env python3
"""probe_dtypes.py — 8-source single-bucket reductions at config B/E shapes
for every dtype/op the configs name (fp32/fp16/bf16 sum at 256 MiB per input,
int64 max and fp8 e4m3/e5m2 sum at 128 MiB), device time per launch and
algorithmic GB/s, one process. Not the bench."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    nbx.load_library()
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    cases = [("f32 sum", 7, 0, 4, 256), ("f16 sum", 6, 0, 2, 256), ("bf16 sum", 9, 0, 2, 256),
             ("i64 max", 4, 2, 8, 128), ("fp8e4m3 sum", 10, 0, 1, 128), ("fp8e5m2 sum", 11, 0, 1, 128),
             ("f32 max", 7, 2, 4, 256), ("f32 avg (premulsum)", 7, 4, 4, 256)]
    for name, dt, redop, esz, mib in cases:
        n = (mib << 20) // esz
        g = torch.Generator(device="cuda").manual_seed(5)
        srcs = []
        for _ in range(8):
            b = torch.randint(0, 256, (mib << 20,), dtype=torch.uint8, device="cuda", generator=g)
            if dt in (10, 11):
                b &= 0x77   # finite codes
            elif dt in (6, 9, 7):
                b = torch.rand(n, device="cuda", generator=g).to({6: torch.float16, 9: torch.bfloat16,
                                                                    7: torch.float32}[dt]).view(torch.uint8)
            srcs.append(b)
        out = torch.empty(mib << 20, dtype=torch.uint8, device="cuda")
        sp = [t.data_ptr() for t in srcs]
        op = nbx.host_to_dev_redop(redop, dt, 8)
        ts = []
        for _ in range(5):
            nbx.reduce_multi([out.data_ptr()], sp, n, dt, op, 8 if redop == 4 else 0, False, st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(10):
                nbx.reduce_multi([out.data_ptr()], sp, n, dt, op, 8 if redop == 4 else 0, False, st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        ts.sort()
        ms = ts[len(ts) // 2]
        print(json.dumps({"case": name, "MiB_per_input": mib, "nsrc": 8, "ms": round(ms, 4),
                          "GBps": round(9 * (mib << 20) / (ms * 1e-3) / 1e9, 1)}), flush=True)
        del srcs, out


if __name__ == "__main__":
    main()
