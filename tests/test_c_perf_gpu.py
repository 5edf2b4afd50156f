"""The nccl-tests style C driver (tests/c/nbx_perf.c, built by build() into
neuronabox-nccl_amd/lib/nbx_perf) against libnbxccl.so on the GPU: an NCCL C
caller (ncclCommInitAll + ncclGroupStart/End, one process driving every rank)
running all_reduce / reduce_scatter / reduce sweeps out-of-place and in-place,
every size checked on the host (#wrong == 0). Ranks share the box's one GPU."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "neuronabox-nccl_amd", "lib", "nbx_perf")


@pytest.mark.parametrize("args", [
    ["-c", "allreduce", "-d", "0,0", "-t", "float", "-o", "sum"],
    ["-c", "allreduce", "-d", "0,0,0", "-t", "half", "-o", "max"],
    ["-c", "allreduce", "-d", "0,0,0,0", "-t", "int32", "-o", "avg"],
    ["-c", "allreduce", "-d", "0,0,0", "-t", "bfloat16", "-o", "avg"],
    ["-c", "reducescatter", "-d", "0,0,0", "-t", "float", "-o", "sum"],
    ["-c", "reducescatter", "-d", "0,0", "-t", "int64", "-o", "min"],
    ["-c", "reduce", "-d", "0,0,0", "-t", "double", "-o", "sum"],
])
def test_nbx_perf_sweep(args):
    assert os.path.exists(EXE), "nbx_perf not built: run __graft_entry__.build()"
    out = subprocess.run([EXE, *args, "-b", "1000", "-e", str(8 << 20), "-f", "8", "-n", "5", "-w", "1"],
                         capture_output=True, text=True, timeout=240)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "Out of bounds values : 0 OK" in out.stdout
    rows = [l for l in out.stdout.splitlines() if l.strip() and not l.startswith("#")]
    assert len(rows) >= 4
