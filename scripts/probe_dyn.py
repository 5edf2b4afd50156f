#!/usr/bin/env python3
"""probe_dyn.py — single-bucket fp32 sums at 256 MiB per input for 1-8
sources (and fp16 at 64 MiB), one process; run once per NBX_DYNAMIC_TILES
setting (0 static, 1 dynamic big tiles, 2 dynamic small tiles too). Not the
bench. Prints one JSON line per case."""
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
    for dt, tdt, mib, nsrcs in ((7, torch.float32, 256, (1, 2, 3, 4, 8)), (6, torch.float16, 64, (2, 8))):
        esz = torch.tensor([], dtype=tdt).element_size()
        n = (mib << 20) // esz
        for nsrc in nsrcs:
            srcs = [torch.rand(n, device="cuda").to(tdt) for _ in range(nsrc)]
            out = torch.empty_like(srcs[0])
            sp = [t.data_ptr() for t in srcs]
            op = nbx.host_to_dev_redop(0, dt, 1)
            ts = []
            for _ in range(5):
                for _ in range(2):
                    nbx.reduce_multi([out.data_ptr()], sp, n, dt, op, 0, False, st.cuda_stream)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(10):
                    nbx.reduce_multi([out.data_ptr()], sp, n, dt, op, 0, False, st.cuda_stream)
                e1.record(st)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 10)
            ts.sort()
            ms = ts[len(ts) // 2]
            print(json.dumps({"dyn": os.environ.get("NBX_DYNAMIC_TILES", "1"), "dtype": str(tdt).split(".")[-1],
                              "nsrc": nsrc, "MiB_per_input": mib, "ms": round(ms, 4),
                              "GBps": round((nsrc + 1) * n * esz / (ms * 1e-3) / 1e9, 1)}), flush=True)
            del srcs, out


if __name__ == "__main__":
    main()
