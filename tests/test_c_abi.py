"""Build and run a plain C program against include/nccl.h + libnbxccl.so
(gcc, -lnbxccl): the drop-in link path INTEGRATION.md describes."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_caller_links_and_runs(nbx, tmp_path):
    libdir = os.path.dirname(nbx.library_path())
    exe = tmp_path / "abi_smoke"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "abi_smoke.c"), "-L", libdir, "-lnbxccl",
                    f"-Wl,-rpath,{libdir}", "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "OK"
