#!/usr/bin/env python3
"""Static check of vector-memory waits in a compiled gfx9 kernel.

The experimental rings of csrc/vcache.hip (CX == 2, LD == 2) and
csrc/wgather.hip (k_wgather_pipe) issue their loads with inline asm.  The
compiler's waitcnt pass does not see those loads, so their `s_waitcnt vmcnt`
are written by hand.  This tool checks the hand-written waits against the
register allocation the compiler actually chose.  It runs a dataflow pass
over the kernel's control-flow graph, built from hipcc `--cuda-device-only -S`
output.

* State: for each VGPR that a vector-memory load may still be writing, the
  smallest number of vector-memory operations that could have been issued
  after that load.  Loads, stores and LDS-DMA all count, since on gfx9 every
  vector-memory operation is counted by vmcnt in issue order.
* At a join, the smallest count from any incoming path is kept.
* `s_waitcnt vmcnt(N)` retires every register whose count is N or more.
* A violation is any instruction that reads or overwrites a register that
  may still be pending.

Compiler-generated code passes by construction, so the tool also checks
itself on the product kernels.

    python tools/vmcnt_check.py kernel.s [symbol-substring ...]
Exit status 1 if any kernel has a violation.
"""
from __future__ import annotations

import re
import sys

VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
VMEM_LOAD = re.compile(r"^(global_load|buffer_load|flat_load|scratch_load)")
VMEM_STORE = re.compile(r"^(global_store|buffer_store|flat_store|scratch_store|global_atomic|buffer_atomic|flat_atomic)")
BRANCH = re.compile(r"^s_(c?branch\w*)\s+(\.?\w+)")


def vregs(text: str) -> set[int]:
    out = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse_kernel(lines: list[str], start: int):
    """Instructions of the function starting at lines[start] (its label), with
    labels; stops at s_endpgm / the function's end."""
    body = []
    for l in lines[start + 1:]:
        s = l.split(";")[0].rstrip()
        t = s.strip()
        if not t:
            continue
        if re.match(r"^\.?L\w+:", t) or re.match(r"^\w+:", t):
            body.append(("label", t[:-1]))
            continue
        if t.startswith("."):
            if t.startswith(".Lfunc_end"):
                break
            continue
        body.append(("ins", t))
    return body


def blocks_of(body):
    """Split into basic blocks: list of (label, [instrs], [successor labels])."""
    blocks, cur, name, n = [], [], "entry", 0
    def close(succ_fall=True):
        nonlocal cur, name
        blocks.append([name, cur, [], succ_fall])
        cur = []
    for kind, t in body:
        if kind == "label":
            if cur or blocks == [] or blocks[-1][0] != name:
                close()
            name = t
            continue
        cur.append(t)
        m = BRANCH.match(t)
        if m or t.startswith("s_endpgm") or t.startswith("s_setpc"):
            uncond = t.startswith("s_branch") or t.startswith("s_endpgm") or t.startswith("s_setpc")
            blocks.append([name, cur, [m.group(2)] if m else [], not uncond])
            cur = []
            n += 1
            name = f"__fall{n}"
    if cur:
        blocks.append([name, cur, [], False])
    # successors: explicit targets + fallthrough to the next block
    for i, b in enumerate(blocks):
        if b[3] and i + 1 < len(blocks):
            b[2].append(blocks[i + 1][0])
    return [b for b in blocks if b[1] or b[2]]


def transfer(state: dict[int, int], ins: str, report=None):
    op = ins.split()[0]
    args = ins[len(op):].strip()
    parts = [p.strip() for p in args.split(",")] if args else []
    if op == "s_waitcnt":
        m = re.search(r"vmcnt\((\d+)\)", ins)
        if m:
            n = int(m.group(1))
            for r in [r for r, a in state.items() if a >= n]:
                del state[r]
        return state
    is_load = bool(VMEM_LOAD.match(op)) and "_lds" not in op and " lds" not in ins
    is_vm = bool(VMEM_LOAD.match(op) or VMEM_STORE.match(op))
    # registers read / written by this instruction
    if is_load:
        dst, src = vregs(parts[0]) if parts else set(), set().union(*(vregs(p) for p in parts[1:])) if len(parts) > 1 else set()
    elif VMEM_STORE.match(op) or op.startswith("ds_write") or op.startswith("ds_add") \
            or op.startswith("s_") or op.startswith("global_load_lds") or op.startswith("buffer_load") and "lds" in ins:
        dst, src = set(), set().union(*(vregs(p) for p in parts)) if parts else set()
    else:
        dst = vregs(parts[0]) if parts else set()
        src = set().union(*(vregs(p) for p in parts[1:])) if len(parts) > 1 else set()
    if report is not None:
        bad_r = src & state.keys()
        # a load may target a register another load is still writing: loads
        # return in issue order, so the younger value lands last
        bad_w = set() if is_load else dst & state.keys()
        if bad_r:
            report.append(f"reads pending v{sorted(bad_r)}: {ins}")
        if bad_w:
            report.append(f"overwrites pending v{sorted(bad_w)}: {ins}")
    for r in list(dst):
        state.pop(r, None)
    if is_vm:
        for r in state:
            state[r] += 1
    if is_load:
        for r in dst:
            state[r] = 0
    return state


def merge(a: dict | None, b: dict) -> dict:
    if a is None:
        return dict(b)
    out = dict(a)
    for r, age in b.items():
        out[r] = min(out.get(r, age), age)
    return out


def check(blocks) -> list[str]:
    idx = {b[0]: i for i, b in enumerate(blocks)}
    ins_state = [None] * len(blocks)
    ins_state[0] = {}
    work = [0]
    while work:
        i = work.pop()
        st = dict(ins_state[i])
        for t in blocks[i][1]:
            st = transfer(st, t)
        for s in blocks[i][2]:
            j = idx.get(s)
            if j is None:
                continue
            m = merge(ins_state[j], st)
            if m != ins_state[j]:
                ins_state[j] = m
                work.append(j)
    report = []
    for i, b in enumerate(blocks):
        if ins_state[i] is None:
            continue
        st = dict(ins_state[i])
        for t in b[1]:
            st = transfer(st, t, report)
    return report


def main(argv):
    path, subs = argv[1], argv[2:]
    lines = open(path).read().splitlines()
    bad = 0
    for k, l in enumerate(lines):
        m = re.match(r"^(_Z\w+):", l)
        if not m or (subs and not any(s in m.group(1) for s in subs)):
            continue
        rep = check(blocks_of(parse_kernel(lines, k)))
        print(f"{m.group(1)[:90]}: {len(rep)} violations")
        for r in rep[:10]:
            print("   ", r)
        bad += bool(rep)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
