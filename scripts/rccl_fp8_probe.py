#!/usr/bin/env python3
"""rccl_fp8_probe.py — RCCL 2.26's one-rank fp8 PreMulSum (librccl's C API via
ctypes) against libnbxccl's on every fp8 code x a set of scalars: prints, per
(format, scalar), every code whose results differ (input, RCCL, ours) and a
count by class. usage: rccl_fp8_probe.py REPO_ROOT"""
import ctypes
import json
import os
import sys

sys.path.insert(0, sys.argv[1])
import torch  # noqa: E402

torch.cuda.set_device(0)
rccl = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"), mode=ctypes.RTLD_LOCAL)
rccl.ncclCommInitAll.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
rccl.ncclRedOpCreatePreMulSum.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
rccl.ncclRedOpDestroy.argtypes = [ctypes.c_int, ctypes.c_void_p]
rccl.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_void_p]
from tests.conftest import load_package  # noqa: E402

nbx = load_package()
nbx.load_library()
rc_comm = ctypes.c_void_p()
assert rccl.ncclCommInitAll(ctypes.byref(rc_comm), 1, (ctypes.c_int * 1)(0)) == 0
comm = nbx.Communicator.init_all([0])[0]
st = torch.cuda.current_stream().cuda_stream
x8 = torch.arange(256, dtype=torch.uint8, device="cuda")
for code, dt in ((10, torch.float8_e4m3fn), (11, torch.float8_e5m2)):
    for f in (0.1, -2.5, 1.0 / 3.0, 1e-3, 3.0, 0.125, 448.0, 2.0 ** -6, 1.0, -1.0):
        sc = torch.tensor([f], dtype=torch.float32).to(dt)
        y = torch.empty_like(x8)
        z = torch.empty_like(x8)
        op = ctypes.c_int()
        assert rccl.ncclRedOpCreatePreMulSum(ctypes.byref(op), ctypes.c_void_p(sc.data_ptr()), code, 1, rc_comm) == 0
        assert rccl.ncclAllReduce(ctypes.c_void_p(x8.data_ptr()), ctypes.c_void_p(y.data_ptr()), 256, code, op.value,
                                  rc_comm, ctypes.c_void_p(st)) == 0
        torch.cuda.synchronize()
        rccl.ncclRedOpDestroy(op.value, rc_comm)
        ours = comm.redop_create_premulsum(sc.data_ptr(), code)
        comm.all_reduce(x8.data_ptr(), z.data_ptr(), 256, code, ours, st)
        torch.cuda.synchronize()
        comm.redop_destroy(ours)
        xs, ys, zs = x8.cpu().tolist(), y.cpu().tolist(), z.cpu().tolist()
        xf = x8.view(dt).float().cpu().tolist()
        scf = float(sc.float())
        rows = [(f"{a:02x}", xf[i], f"{b:02x}", f"{c:02x}") for i, (a, b, c) in enumerate(zip(xs, ys, zs)) if b != c]
        print(json.dumps({"type": code, "scalar": f, "scalar_in_type": scf, "n_diff": len(rows), "diff": rows}))
comm.destroy()
