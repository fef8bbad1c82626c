"""Compare the gfx950 machine code of two builds of libosc_batch.so kernel by kernel.

    python tools/isa_compare.py old.so new.so [--strip REGEX] [substring ...]

--strip REGEX rewrites the OLD build's kernel names, each match of REGEX replaced by its first
group (or removed if it has none): a dropped template argument renames every instantiation
without changing its code.

Used to show that a source change (pruning dead compile-time variants, adding an opt-in model
instantiation) leaves the product kernels' instruction streams untouched: a kernel whose
disassembly (addresses and encodings stripped) is identical computes bitwise-identical results.
Exit status 1 when a kernel present in both differs; kernels present in only one are listed.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def kernels(so: str) -> dict[str, str]:
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "fat.bin"), os.path.join(td, "k.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", so,
                        os.path.join(td, "junk")], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        f"--input={fat}", f"--targets={TARGET}", f"--output={co}"], check=True)
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn",
                              "--no-leading-addr", co], check=True, capture_output=True,
                             text=True).stdout
    out: dict[str, list[str]] = {}
    cur = None
    for line in dis.splitlines():
        m = re.match(r"^<(.+)>:$", line.strip())
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is None:
            continue
        s = line.split("//")[0].strip()
        if s:
            out[cur].append(s)
    return {k: "\n".join(v) for k, v in out.items()}


def main(argv: list[str]) -> int:
    a, b = kernels(argv[1]), kernels(argv[2])
    subs = argv[3:]
    if subs[:1] == ["--strip"]:
        rx = re.compile(subs[1])
        a = {rx.sub(r"\1" if rx.groups else "", k): v for k, v in a.items()}
        subs = subs[2:]
    keep = lambda k: not subs or any(s in k for s in subs)
    rc = 0
    for k in sorted(set(a) | set(b)):
        if not keep(k):
            continue
        if k not in a:
            print(f"new      {k}")
        elif k not in b:
            print(f"removed  {k}")
        elif a[k] != b[k]:
            print(f"DIFFERS  {k}  ({a[k].count(chr(10)) + 1} -> {b[k].count(chr(10)) + 1} lines)")
            rc = 1
        else:
            print(f"same     {k}")
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv))
