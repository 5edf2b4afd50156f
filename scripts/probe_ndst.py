#!/usr/bin/env python3
"""probe_ndst.py — nbxReduceMulti time vs destination count (1, 2, 8) for a
few (type, op, nSrcs) shapes, 64 MiB per buffer, one GPU. Prints JSON lines."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from __graft_entry__ import _load_package
    nbx = _load_package()
    nbx.load_library()
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 64 << 20
    bufs = [torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(16)]
    for dt, op, eb, name in ((4, 2, 8, "int64 max"), (7, 0, 4, "f32 sum"), (10, 0, 1, "fp8 sum"), (2, 2, 4, "int32 max")):
        devop = nbx.host_to_dev_redop(op, dt, 2)
        for nsrc in (2, 8):
            for ndst in (1, 2, 8):
                srcs = [b.data_ptr() for b in bufs[:nsrc]]
                dsts = [b.data_ptr() for b in bufs[8:8 + ndst]]
                cnt = nbytes // eb
                f = lambda: nbx.reduce_multi(dsts, srcs, cnt, dt, devop, 0, False, st)
                for _ in range(3):
                    f()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(20):
                    f()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) * 1e3 / 20
                print(json.dumps({"what": name, "nsrc": nsrc, "ndst": ndst, "ms": round(ms, 4),
                                  "GBps": round((nsrc + ndst) * nbytes / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
