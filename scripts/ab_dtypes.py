#!/usr/bin/env python3
"""ab_dtypes.py — in-process A/B of several builds of libnbxccl.so on the
configs' 8-source single-bucket shapes for every dtype/op the configs name
(fp32/fp16/bf16 sum at 256 MiB per input, int64 max and fp8 e4m3/e5m2 sum at
128 MiB, fp32 max): same buffers, same stream, builds interleaved per round,
median device time per launch (HIP events around 10 back-to-back calls) and
algorithmic GB/s per build; outputs compared bit for bit across builds.
--bpc 0,2 runs every build at each workgroups-per-CU knob (nbxSetLaunchConfig;
0 = the build's default) as separate contestants.
usage: ab_dtypes.py a.so b.so [...] [--rounds R] [--cases f32,fp8e4m3,...] [--bpc 0,2]"""
import ctypes
import json
import sys

import torch


class DevRedOpFull(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("scalarArgIsPtr", ctypes.c_int32), ("scalarArg", ctypes.c_uint64)]


CASES = {   # name: (ncclDataType_t, ncclRedOp_t, element size, MiB per input)
    "f32": (7, 0, 4, 256), "f16": (6, 0, 2, 256), "bf16": (9, 0, 2, 256), "i64max": (4, 2, 8, 128),
    "fp8e4m3": (10, 0, 1, 128), "fp8e5m2": (11, 0, 1, 128), "f32max": (7, 2, 4, 256),
    "i32max": (2, 2, 4, 256), "u32min": (3, 3, 4, 256), "i8max": (0, 2, 1, 256), "u64min": (5, 3, 8, 128),
    "u8min": (1, 3, 1, 256), "u8sum": (1, 0, 1, 256), "i8prod": (0, 1, 1, 256), "i32prod": (2, 1, 4, 256),
    "i64prod": (4, 1, 8, 128), "i64sum": (4, 0, 8, 128), "i32sum": (2, 0, 4, 256),
    "i8avg": (0, 4, 1, 256), "u32avg": (3, 4, 4, 256), "i64avg": (4, 4, 8, 128),
    "f16max": (6, 2, 2, 256), "bf16max": (9, 2, 2, 256), "f64sum": (8, 0, 8, 256), "f64max": (8, 2, 8, 256),
    "f16prod": (6, 1, 2, 256), "f32prod": (7, 1, 4, 256), "bf16avg": (9, 4, 2, 256), "f32avg": (7, 4, 4, 256),
    "fp8max": (10, 2, 1, 128), "fp8e5min": (11, 3, 1, 128), "fp8prod": (10, 1, 1, 128), "fp8avg": (10, 4, 1, 128),
}


def load(path):
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    f = lib.nbxReduceMulti
    f.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                  ctypes.c_size_t, ctypes.c_int, DevRedOpFull, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    f.restype = ctypes.c_int
    h = lib.nbxHostToDevRedOp
    h.argtypes = [ctypes.POINTER(DevRedOpFull), ctypes.c_int, ctypes.c_int, ctypes.c_int]
    h.restype = ctypes.c_int
    lc = lib.nbxSetLaunchConfig
    lc.argtypes = [ctypes.c_int, ctypes.c_int]
    lc.restype = ctypes.c_int
    return f, h, lc


def main():
    argv = sys.argv[1:]
    paths = [a for a in argv if a.endswith(".so")]
    rounds = int(argv[argv.index("--rounds") + 1]) if "--rounds" in argv else 5
    names = argv[argv.index("--cases") + 1].split(",") if "--cases" in argv else list(CASES)
    bpcs = [int(x) for x in argv[argv.index("--bpc") + 1].split(",")] if "--bpc" in argv else [0]
    loaded = [load(p) for p in paths]
    libs = [(f, h, lc, b) for (f, h, lc) in loaded for b in bpcs]
    labels = [f"{p}@bpc{b}" if len(bpcs) > 1 else p for p in paths for b in bpcs]
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    for name in names:
        dt, redop, esz, mib = CASES[name]
        n = (mib << 20) // esz
        g = torch.Generator(device="cuda").manual_seed(5)
        srcs = []
        for _ in range(8):
            if dt in (6, 9, 7, 8):
                b = torch.rand(n, device="cuda", generator=g).to({6: torch.float16, 9: torch.bfloat16,
                                                                    7: torch.float32, 8: torch.float64}[dt]).view(torch.uint8)
            else:
                b = torch.randint(0, 256, (mib << 20,), dtype=torch.uint8, device="cuda", generator=g)
                if dt in (10, 11):
                    b &= 0x77   # finite codes
            srcs.append(b)
        # ONE output buffer for every contestant: the output's placement alone
        # moved byte-identical kernels by up to 9 % (profiles/r5/ab_swar8_r5i.jsonl,
        # scripts/sweep_out_placement.hip); each contestant's first result is
        # kept for the bit-for-bit comparison
        out = torch.empty(mib << 20, dtype=torch.uint8, device="cuda")
        outs = [None for _ in libs]
        S = (ctypes.c_void_p * 8)(*[t.data_ptr() for t in srcs])
        Ds = [(ctypes.c_void_p * 1)(out.data_ptr()) for _ in libs]
        ops = []
        for f, h, _, _ in libs:
            op = DevRedOpFull()
            assert h(ctypes.byref(op), redop, dt, 8) == 0
            ops.append(op)
        times = [[] for _ in libs]
        for _ in range(rounds):
            for k, (f, _, lc, b) in enumerate(libs):
                assert lc(b, 0) == 0
                for _ in range(3):
                    assert f(Ds[k], 1, S, 8, n, dt, ops[k], 0, 0, st.cuda_stream) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(10):
                    f(Ds[k], 1, S, 8, n, dt, ops[k], 0, 0, st.cuda_stream)
                e1.record(st)
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / 10)
                if outs[k] is None:
                    outs[k] = out.clone()
        same = all(torch.equal(outs[0], o) for o in outs[1:])
        row = {"case": name, "MiB_per_input": mib, "nsrc": 8, "identical": same}
        for k, p in enumerate(labels):
            ts = sorted(times[k])
            ms = ts[len(ts) // 2]
            row[p] = {"ms": round(ms, 4), "GBps": round(9 * (mib << 20) / (ms * 1e-3) / 1e9, 1)}
        print(json.dumps(row), flush=True)
        del srcs, outs, out


if __name__ == "__main__":
    main()
