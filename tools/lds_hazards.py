#!/usr/bin/env python3
"""Static check of the hand-scheduled LDS reads in the gfx950 code objects.

The trunk kernels read their MFMA fragments with inline-asm `ds_read_b128` and wait for them with
inline-asm `s_waitcnt lgkmcnt(N)`.  The compiler does not know these loads are asynchronous: it
treats the asm's output registers as written when the asm issues.  A register whose load is still in
flight can therefore be reused -- a loop-exit copy, an epilogue address -- and the late LDS return
then overwrites the live value.  That happens only when LDS is slow (several blocks per CU), so
tests at one block per CU pass; conv3x3_v7 with 128-row tiles gave wrong outputs or an illegal
address at two or three blocks per CU before the loops got their drains.

This runs a dataflow over every kernel's control-flow graph, keeps the queue of outstanding LDS /
scalar-memory operations that `s_waitcnt lgkmcnt(N)` retires oldest first, and reports every
non-LDS instruction that reads or writes a register an outstanding `ds_read` still targets.  (Two
LDS loads into the same register are not reported: LDS returns in order.)

Usage: python3 tools/lds_hazards.py [object ...]   (default: the in-tree build's kernel objects)
Exit status 1 when any kernel has a hazard."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
DEFAULT = ["conv_v7.o", "conv_bf16.o", "smallnet.o", "net_kernels.o", "tree_kernels.o", "engine.o", "dataset.o"]
BRANCHES = {"s_branch", "s_cbranch_scc0", "s_cbranch_scc1", "s_cbranch_vccz", "s_cbranch_vccnz",
            "s_cbranch_execz", "s_cbranch_execnz"}
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def vregs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return frozenset(out)


def device_disasm(obj):
    """gfx950 code object of a hipcc-built host object -> llvm-objdump text"""
    with open(obj, "rb") as f:
        head = f.read(20)
    if head[:4] == b"\x7fELF" and int.from_bytes(head[18:20], "little") == 0xE0:   # already AMDGPU
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", obj], check=True, capture_output=True, text=True).stdout
    with tempfile.TemporaryDirectory() as td:
        fb, dev = os.path.join(td, "fb.bin"), os.path.join(td, "dev.o")
        if subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(td, "h.o")],
                          capture_output=True).returncode or not os.path.exists(fb) or not os.path.getsize(fb):
            return ""                                     # no device code
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], check=True,
                       capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", dev], check=True, capture_output=True,
                              text=True).stdout


def split_kernels(text):
    funcs, cur = {}, None
    for line in text.split("\n"):
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
        elif cur:
            m = re.match(r"\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", line)
            if m:
                funcs[cur].append((int(m.group(3), 16), m.group(1), m.group(2)))
    return funcs


def scan(ins):
    """hazards of one kernel: [(index, op, operands, registers, index of the ds_read)]

    Forward dataflow to a fixpoint.  The state at an instruction is the queue of outstanding
    lgkm operations, youngest first; each slot holds the (register, ds_read index) pairs its
    operation will still write (empty for writes and scalar loads).  Paths merge slot by slot
    (union), which over-approximates but keeps the walk linear in the code size."""
    at = {a: i for i, (a, _, _) in enumerate(ins)}
    state = {0: ()}
    work = [0]
    found = {}

    def merge(i, st):
        old = state.get(i)
        if old is None:
            state[i] = st
            work.append(i)
            return
        n = max(len(old), len(st))
        m = tuple((old[k] if k < len(old) else frozenset()) | (st[k] if k < len(st) else frozenset()) for k in range(n))
        if m != old:
            state[i] = m
            work.append(i)

    while work:
        i = work.pop()
        pend = state[i]
        a, op, ops = ins[i]
        succ = [i + 1]
        if op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", ops)
            if m:
                pend = pend[:int(m.group(1))]
        elif op == "s_endpgm":
            succ = []
        elif op in BRANCHES:
            off = int(ops.split()[0])
            off = off - 65536 if off >= 32768 else off
            tgt = at.get(a + 4 + 4 * off)
            succ = ([tgt] if tgt is not None else []) + ([] if op == "s_branch" else [i + 1])
        elif op.startswith("ds_") or op.startswith("s_load") or op.startswith("s_buffer_load"):
            returns = op.startswith(("ds_read", "ds_bpermute", "ds_permute", "ds_swizzle")) or "_rtn" in op
            dst = frozenset((r, i) for r in vregs(ops.split(",")[0])) if returns else frozenset()
            pend = ((dst,) + pend)[:16]
        elif not op.startswith("s_"):
            r = vregs(ops)
            for slot in pend:
                for reg, j in slot:
                    if reg in r:
                        found.setdefault((i, j), set()).add(reg)
        for k in succ:
            if k < len(ins):
                merge(k, pend)
    return [(i, ins[i][1], ins[i][2], sorted(regs), j) for (i, j), regs in sorted(found.items())]


def main(argv):
    objs = argv or [os.path.join(ROOT, "alphazero-multi-game_amd", "build", o) for o in DEFAULT]
    total = 0
    for obj in objs:
        if not os.path.exists(obj):
            print(f"{obj}: missing")
            continue
        kernels = split_kernels(device_disasm(obj))
        bad = 0
        for name, ins in kernels.items():
            hz = scan(ins)
            if hz:
                bad += 1
                total += len(hz)
                dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
                print(f"{os.path.basename(obj)}: {dn}: {len(hz)} hazards")
                for i, op, ops, regs, j in hz[:4]:
                    print(f"    {op} {ops[:60]}  touches v{regs} of the ds_read at +{ins[j][0] - ins[0][0]:#x}")
        print(f"{os.path.basename(obj)}: {len(kernels)} kernels, {bad} with hazards")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
