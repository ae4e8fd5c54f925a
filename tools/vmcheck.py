#!/usr/bin/env python3
"""Static check of untracked (inline-asm) vector loads in a disassembled kernel.

The fused front end issues its tile prefetch as inline-asm global_load_dwordx4
(fir_parts.hpp ldg4_async) and waits for it itself, so hipcc's waitcnt pass does
not protect those registers.  This walks the kernel's control-flow graph and
reports any instruction that reads or writes a VGPR while a dwordx4 load into
it may still be in flight (no s_waitcnt vmcnt(N) since with N small enough).

Dataflow state: for each pending VGPR, the minimum number of dwordx4 loads
issued after it on any path (its "age"); s_waitcnt vmcnt(N) retires ages >= N.
Stores and other VMEM ops are ignored, which only keeps registers pending
longer (conservative).

usage: llvm-objdump -d --no-show-raw-insn k.co > k.s; vmcheck.py k.s [kernel-substring]
"""
import re
import sys

INS = re.compile(r"^\s+(\w+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):")
TGT = re.compile(r"<[^>]*\+0x([0-9a-f]+)>")
LABEL = re.compile(r"^([0-9a-f]+) <(\S+)>:$")


def vregs(text):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", text):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def kernels(path, want):
    cur, body = None, []
    for line in open(path):
        m = LABEL.match(line.strip())
        if m:
            if cur and (want is None or want in cur):
                yield cur, body
            cur, body = m.group(2), []
            continue
        body.append(line)
    if cur and (want is None or want in cur):
        yield cur, body


def check(name, lines):
    insts = []  # (offset, op, operands, raw target offset or None)
    base = None
    for line in lines:
        m = INS.match(line)
        if not m:
            continue
        op, ops, addr = m.group(1), m.group(2), int(m.group(3), 16)
        if base is None:
            base = addr
        t = TGT.search(line)
        insts.append((addr - base, op, ops, int(t.group(1), 16) if t and op.startswith("s_") and "branch" in op else None))
    if not insts:
        return 0
    idx = {off: i for i, (off, *_r) in enumerate(insts)}
    # successors per instruction index
    succ = []
    for i, (off, op, ops, tgt) in enumerate(insts):
        s = []
        if op == "s_endpgm":
            pass
        elif op == "s_branch":
            s.append(idx.get(tgt))
        else:
            if op.startswith("s_cbranch"):
                s.append(idx.get(tgt))
            if i + 1 < len(insts):
                s.append(i + 1)
        succ.append([x for x in s if x is not None])
    state = [None] * len(insts)  # dict reg -> age at entry
    state[0] = {}
    work = [0]
    problems = {}
    while work:
        i = work.pop()
        cur = dict(state[i])
        off, op, ops, _t = insts[i]
        parts = [p.strip() for p in ops.split(",")] if ops else []
        if op.startswith("s_waitcnt"):
            m = re.search(r"vmcnt\((\d+)\)", ops)
            if m:
                n = int(m.group(1))
                cur = {r: a for r, a in cur.items() if a < n}
        elif op == "global_load_dwordx4":
            addr = vregs(",".join(parts[1:]))
            if addr & set(cur):
                problems.setdefault(off, f"address of {op} {ops} still in flight")
            cur = {r: a + 1 for r, a in cur.items()}
            for r in vregs(parts[0]):
                cur[r] = 0
        elif op.startswith("v_") or op.startswith("ds_") or op.startswith("global_") or op.startswith("buffer_") \
                or op.startswith("flat_"):
            touched = vregs(ops)
            bad = touched & set(cur)
            if bad:
                problems.setdefault(off, f"{op} {ops} touches v{sorted(bad)[:4]} in flight")
        for j in succ[i]:
            if state[j] is None:
                state[j] = dict(cur)
                work.append(j)
            else:
                merged = dict(state[j])
                changed = False
                for r, a in cur.items():
                    if r not in merged or a < merged[r]:
                        merged[r] = a
                        changed = True
                if changed:
                    state[j] = merged
                    work.append(j)
    for off in sorted(problems):
        print(f"  +0x{off:x}: {problems[off]}")
    print(f"{name}: {len(problems)} hazard(s)")
    return len(problems)


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else None
    total = sum(check(n, b) for n, b in kernels(path, want))
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
