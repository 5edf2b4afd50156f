#!/usr/bin/env python3
"""disasm_kernel.py — print the gfx950 disassembly of one kernel of
libnbxccl.so (exact mangled name, or a unique substring), plus an opcode
histogram with --hist. usage: disasm_kernel.py NAME [--hist] [--so PATH]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_objects(so):
    tmp = tempfile.mkdtemp()
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", so, os.devnull], check=True)
    blob = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
    for i, s in enumerate(starts):
        b, e = os.path.join(tmp, f"b{i}.bin"), os.path.join(tmp, f"b{i}.elf")
        open(b, "wb").write(blob[s:starts[i + 1] if i + 1 < len(starts) else len(blob)])
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle", f"--input={b}", f"--output={e}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(e) > 0:
            yield e


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    so = os.path.join(ROOT, "neuronabox-nccl_amd", "lib", "libnbxccl.so")
    if "--so" in sys.argv:
        so = sys.argv[sys.argv.index("--so") + 1]
        args = [a for a in args if a != so]
    name = args[0]
    for e in code_objects(so):
        d = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", e], capture_output=True,
                           text=True).stdout
        for m in re.finditer(r"\n[0-9a-f]+ <([^>]+)>:\n", d):
            if m.group(1) == name or name in m.group(1):
                nxt = re.search(r"\n[0-9a-f]+ <[^>]+>:\n", d[m.end():])
                body = d[m.end(): m.end() + nxt.start() if nxt else len(d)]
                ops = re.findall(r"^\s+([a-z_0-9]+)", body, re.M)
                print(f"# {m.group(1)}: {len(ops)} instructions")
                if "--hist" in sys.argv:
                    from collections import Counter
                    for op, c in Counter(ops).most_common(25):
                        print(f"{c:6d} {op}")
                else:
                    print(body)
                return 0
    print("kernel not found", file=sys.stderr)
    return 1


if __name__ == "__main__":
    sys.exit(main())
