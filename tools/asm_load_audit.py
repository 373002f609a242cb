"""Audit inline-asm VGPR loads in a hipcc -S listing: for every `buffer_load_dwordx4 v[a:b]` emitted inside an
;;#ASMSTART block, check that no instruction touches v[a..b] while the load is outstanding. Every vector-memory
instruction in the listing (asm or compiler: loads, LDS DMA, stores) is tracked in program order; an
`s_waitcnt vmcnt(N)` retires all but the N youngest.

Control flow: forward branches are followed as a dataflow over the listing's labels. A conditional branch
(`s_cbranch_*`) sends the current state to its target; an `s_branch` sends it there and makes the fall-through
unreachable; at a label the incoming states are merged (a load stays outstanding if it is outstanding on ANY incoming
path). So a wait that only some waves execute -- e.g. inside a wave-dependent `if` -- does not count for the code after
the branch joins (the hazard class of the round-4 illegal-address fault). Backward branches (loops) are not followed:
at a loop back-edge the outstanding set carries over as in the first iteration.
Usage: asm_load_audit.py file.s [kernel-substring]"""
import re
import sys


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def uses(line):
    ops = line.split(None, 1)
    if len(ops) < 2:
        return set()
    s = set()
    for t in re.split(r"[,\s]+", ops[1]):
        s |= regs(t.strip())
    return s


def merge(a, b):
    """Union of two outstanding lists (entries: (dest regs, line index)), ordered by issue (line index)."""
    if a is None:
        return b
    if b is None:
        return a
    d = {e[1]: e for e in a}
    d.update({e[1]: e for e in b})
    return [d[k] for k in sorted(d)]


def audit(name, lines):
    bad = 0
    labels = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(\.L\w+):", l.strip())
        if m:
            labels[m.group(1)] = i
    incoming = {}            # label -> merged state of the branches to it
    pending = []             # outstanding vector-memory ops: (dest regs, line index); None: unreachable
    inasm = False
    nload = 0
    for i, l in enumerate(lines):
        t = l.strip()
        m = re.match(r"^(\.L\w+):", t)
        if m:
            pending = merge(pending, incoming.pop(m.group(1), None))
            if pending is None:
                pending = []   # reached only by a backward branch (loop header): treat as straight-line
            continue
        if t.startswith(";;#ASMSTART"):
            inasm = True
            continue
        if t.startswith(";;#ASMEND"):
            inasm = False
            continue
        if not t or t.startswith((";", ".")):
            continue
        if pending is None:    # dead code after an unconditional branch until the next label
            continue
        op = t.split()[0]
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = t.split()[1] if len(t.split()) > 1 else ""
            if labels.get(tgt, -1) > i:   # forward: the target sees this state
                incoming[tgt] = merge(incoming.get(tgt), list(pending))
            if op == "s_branch":
                pending = None
            continue
        if inasm and op == "buffer_load_dwordx4":
            pending.append((regs(t.split()[1].rstrip(",")), i))
            nload += 1
            continue
        if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
            pending.append((set(), i))
        if op == "s_waitcnt" and "vmcnt" in t:
            n = int(re.search(r"vmcnt\((\d+)\)", t).group(1))
            pending = pending[len(pending) - n:] if n < len(pending) else pending
            continue
        u = uses(t)
        for rs, li in pending:
            if u & rs:
                bad += 1
                print(f"{name}: line {i}: '{t}' touches v{sorted(u & rs)} of the asm load at line {li} before its wait")
    print(f"{name}: {nload} asm loads audited")
    return bad


def main():
    src = open(sys.argv[1]).read()
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    bad = 0
    for m in re.finditer(r"^(_Z\w+):.*\n", src, re.M):
        name = m.group(1)
        if want not in name:
            continue
        end = src.index(".Lfunc_end", m.end())
        bad += audit(name, src[m.end():end].split("\n"))
    print("BAD" if bad else "OK")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
