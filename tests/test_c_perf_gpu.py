"""The nccl-tests style C driver (tests/c/nbx_perf.c, built by build() into
neuronabox-nccl_amd/lib/nbx_perf) against libnbxccl.so on the GPU: an NCCL C
caller running all_reduce / reduce_scatter / reduce sweeps out-of-place and
in-place, every size checked on the host (#wrong == 0) — one process driving
every rank (ncclCommInitAll + ncclGroupStart/End) and one process per rank
(-p 1: fork + ncclCommInitRank). Ranks share the box's one GPU."""
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
    # -m: 6 independent operations per group (the clique's batched exchange)
    ["-c", "allreduce", "-d", "0,0,0", "-t", "half", "-o", "sum", "-m", "6"],
    ["-c", "reducescatter", "-d", "0,0", "-t", "int32", "-o", "avg", "-m", "4"],
    ["-c", "reduce", "-d", "0,0,0", "-t", "float", "-o", "max", "-m", "3"],
])
def test_nbx_perf_sweep(args):
    _run(args)


# one process per rank (-p 1): the multi-process communicator; sizes 1 KB .. 8 MB
# cross LL, LL128 one-shot, LL128 two-shot and Simple
@pytest.mark.parametrize("args", [
    ["-p", "1", "-c", "allreduce", "-d", "0,0", "-t", "float", "-o", "sum"],
    ["-p", "1", "-c", "allreduce", "-d", "0,0,0,0", "-t", "bfloat16", "-o", "max"],
    ["-p", "1", "-c", "allreduce", "-d", "0,0,0", "-t", "int32", "-o", "avg"],
    ["-p", "1", "-c", "reducescatter", "-d", "0,0,0", "-t", "float", "-o", "sum"],
    ["-p", "1", "-c", "reduce", "-d", "0,0,0", "-t", "half", "-o", "sum"],
    ["-p", "1", "-c", "allreduce", "-d", "0,0", "-t", "float", "-o", "sum", "-m", "3"],
])
def test_nbx_perf_multiprocess(args):
    env = dict(os.environ, NBX_LL128_MAX_GRID="16", NBX_LL_MAX_GRID="64", NBX_TIMEOUT_SEC="60",
               NBX_BOOTSTRAP_TIMEOUT="60")   # ranks share the one GPU: keep spinning grids co-resident
    _run(args, env)


def _run(args, env=None):
    assert os.path.exists(EXE), "nbx_perf not built: run __graft_entry__.build()"
    out = subprocess.run([EXE, *args, "-b", "1000", "-e", str(8 << 20), "-f", "8", "-n", "5", "-w", "1"],
                         capture_output=True, text=True, timeout=240, env=env)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "Out of bounds values : 0 OK" in out.stdout
    rows = [l for l in out.stdout.splitlines() if l.strip() and not l.startswith("#")]
    assert len(rows) >= 4
