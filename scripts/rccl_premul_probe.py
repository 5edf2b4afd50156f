#!/usr/bin/env python3
"""rccl_premul_probe.py — the test_rccl_corroboration_gpu.py child as a script
that prints every mismatch (diagnosis). usage: rccl_premul_probe.py REPO_ROOT
(env RANK=0 WORLD_SIZE=1 MASTER_ADDR / MASTER_PORT set)."""

import json, sys
sys.path.insert(0, sys.argv[1])
import torch
import torch.distributed as dist
import bench
bench.init_process_group("nccl", 0, 1, 0)   # before any other GPU call of this process
torch.cuda.set_device(0)
from tests.conftest import load_package
nbx = load_package()
nbx.load_library()
comm = nbx.Communicator.init_all([0])[0]    # a one-rank communicator of libnbxccl
st = torch.cuda.current_stream().cuda_stream
out = []
# (torch dispatches its NCCL pre-multiply scalar over float / half / double
# only: "expected scalar type Float but found BFloat16" for bf16)
for dt, code in ((torch.float16, 6), (torch.float32, 7), (torch.float64, 8)):
    g = torch.Generator(device="cuda").manual_seed(11)
    x = (torch.randn(1 << 16, generator=g, device="cuda", dtype=torch.float64) * 3).to(dt)
    fi = torch.finfo(dt)
    sp = torch.tensor([float("inf"), -float("inf"), float("nan"), 0.0, -0.0, fi.tiny, -fi.tiny, fi.tiny / 4,
                       fi.max, -fi.max, fi.eps, 1.0, -1.0, 2.0 ** -20], dtype=torch.float64, device="cuda").to(dt)
    x = torch.cat([x, sp])
    n = x.numel()
    for f in (0.1, 1.0 / 3.0, -2.5, 1e-3, 3.0, 0.125, 1.0 / 7.0, 1e-6):
        ft = torch.tensor([f], dtype=dt, device="cuda")
        y = x.clone()
        dist.all_reduce(y, op=dist._make_nccl_premul_sum(ft))
        sc = ft.cpu()                              # the same scalar bits, host-immediate for libnbxccl
        op = comm.redop_create_premulsum(sc.data_ptr(), code)
        z = torch.full_like(x, 7.0)
        comm.all_reduce(x.data_ptr(), z.data_ptr(), n, code, op, st)
        torch.cuda.synchronize()
        comm.redop_destroy(op)
        iy = y.view({2: torch.int16, 4: torch.int32, 8: torch.int64}[x.element_size()])
        iz = z.view(iy.dtype)
        both_nan = torch.isnan(y) & torch.isnan(z)
        diff = ((iy != iz) & ~both_nan).nonzero().flatten()
        out.append({"dtype": str(dt), "factor": f, "n": n, "mismatches": int(diff.numel()),
                    "first": [[float(x[i]), float(y[i]), float(z[i]), hex(int(iy[i]) & 0xffffffffffffffff), hex(int(iz[i]) & 0xffffffffffffffff)] for i in diff[:12].tolist()]})
comm.destroy()
dist.destroy_process_group()
print("RESULT " + json.dumps(out), flush=True)
