#!/usr/bin/env python3
"""Static check of the LDS-DMA stage hand-off ("A stage hand-off race, fixed").

A wave's `global_load_lds` pieces are counted by vmcnt only, and a workgroup barrier does not
wait for them: before every `s_barrier` that a pending LDS-DMA can reach, the wave must have
executed an `s_waitcnt` with vmcnt(0) (fracenc_mfma.hip stage_barrier()).  This disassembles
the gfx950 code object of a library (or a code object file) and runs a forward data-flow
over each kernel's control-flow graph: state "DMA pending" is set by an LDS-DMA instruction,
cleared by `s_waitcnt vmcnt(0)`, and merged over branches; an `s_barrier` reached in that state
is a violation.

usage: tools/lds_dma_check.py LIB_OR_CODE_OBJECT [KERNEL_REGEX]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")
INSN = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):")
TARGET = re.compile(r"<(.+?)\+0x([0-9a-f]+)>")
DMA_OP = re.compile(r"^(global_load_lds|buffer_load_)")


def is_dma(op: str, line: str) -> bool:
    """An LDS-DMA load: global_load_lds_*, or a buffer_load_* with the lds modifier."""
    m = DMA_OP.match(op)
    return bool(m) and (op.startswith("global_load_lds") or re.search(r"\blds\b", line.split("//")[0]) is not None)


def code_object(path: str, workdir: str) -> str:
    """The gfx950 code object inside a hipcc-built shared library (or `path` itself)."""
    with open(path, "rb") as f:
        head = f.read(4)
    if head != b"\x7fELF":
        raise ValueError(f"{path}: not an ELF file")
    sections = subprocess.run(["objdump", "-h", path], capture_output=True, text=True, check=True).stdout
    if ".hip_fatbin" not in sections:
        return path  # already a device code object
    fat = os.path.join(workdir, "fatbin.bin")
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", path, os.path.join(workdir, "host.o")],
                   check=True, capture_output=True)
    co = os.path.join(workdir, "gfx950.co")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
    return co


def disassemble(co: str) -> dict[str, list[tuple[int, str, str]]]:
    """{symbol: [(address, mnemonic, operands+comment)]} of every function in the code object."""
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", "-C", co], capture_output=True,
                         text=True, check=True).stdout
    funcs: dict[str, list] = {}
    cur = None
    for line in out.splitlines():
        m = FUNC.match(line)
        if m:
            cur = funcs.setdefault(m.group(2), [])
            continue
        m = INSN.match(line)
        if m and cur is not None:
            cur.append((int(m.group(3), 16), m.group(1), line))
    return funcs


def violations(insns: list[tuple[int, str, str]]) -> list[str]:
    """Barriers a pending LDS-DMA can reach without an intervening s_waitcnt vmcnt(0)."""
    if not insns:
        return []
    base = insns[0][0]
    index = {a: i for i, (a, _, _) in enumerate(insns)}
    n = len(insns)

    def succ(i):
        _, op, line = insns[i]
        if op == "s_endpgm":
            return []
        nxt = [i + 1] if i + 1 < n else []
        if op.startswith("s_branch") or op.startswith("s_cbranch"):
            m = TARGET.search(line)
            tgt = index.get(base + int(m.group(2), 16)) if m else None
            if tgt is None:
                raise ValueError(f"unresolved branch: {line}")
            return [tgt] if op.startswith("s_branch") else [tgt] + nxt
        if op.startswith("s_setpc") or op.startswith("s_swappc"):
            raise ValueError(f"indirect control flow: {line}")
        return nxt

    pending_in = [False] * n
    seen = [False] * n
    work = [0]
    seen[0] = True
    bad = set()
    while work:
        i = work.pop()
        p = pending_in[i]
        _, op, line = insns[i]
        if op == "s_barrier" and p:
            bad.add(i)
        if is_dma(op, line):
            p = True
        elif op == "s_waitcnt" and re.search(r"\bvmcnt\(0\)", line):
            p = False
        for j in succ(i):
            if not seen[j] or (p and not pending_in[j]):
                seen[j] = True
                pending_in[j] = pending_in[j] or p
                work.append(j)
    return [f"{insns[i][2].strip()}" for i in sorted(bad)]


def check(path: str, kernel_regex: str = ".*") -> tuple[dict[str, list[str]], list[str]]:
    """({kernel: violations} for every matching kernel that issues LDS-DMA, [those kernels])."""
    with tempfile.TemporaryDirectory() as td:
        funcs = disassemble(code_object(path, td))
    rx = re.compile(kernel_regex)
    res, checked = {}, []
    for name, insns in funcs.items():
        if not rx.search(name) or not any(is_dma(op, line) for _, op, line in insns):
            continue
        checked.append(name)
        v = violations(insns)
        if v:
            res[name] = v
    return res, checked


if __name__ == "__main__":
    bad, checked = check(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ".*")
    print(f"{len(checked)} kernels with LDS-DMA checked")
    for k, v in bad.items():
        print(f"VIOLATION {k}:")
        for line in v:
            print("   ", line)
    sys.exit(1 if bad else 0)
