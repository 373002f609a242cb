"""Audit inline-asm VGPR loads in a hipcc -S listing: for every `buffer_load_dwordx4 v[a:b]` emitted inside an
;;#ASMSTART block, check that no instruction touches v[a..b] while the load is outstanding. Every vector-memory
instruction in the listing (asm or compiler: loads, LDS DMA, stores) is tracked in program order; an
`s_waitcnt vmcnt(N)` retires all but the N youngest. The listing is scanned linearly (straight-line unrolled bodies;
at a loop back-edge the outstanding set carries over as in the first iteration). Usage:
asm_load_audit.py file.s [kernel-substring]"""
import re, sys

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

src = open(sys.argv[1]).read()
want = sys.argv[2] if len(sys.argv) > 2 else ""
bad = 0
for m in re.finditer(r"^(_Z\w+):.*\n", src, re.M):
    name = m.group(1)
    if want not in name:
        continue
    end = src.index(".Lfunc_end", m.end())
    lines = src[m.end():end].split("\n")
    inasm = False
    pending = []   # (dest regs, line index)
    nload = 0
    for i, l in enumerate(lines):
        t = l.strip()
        if t.startswith(";;#ASMSTART"):
            inasm = True; continue
        if t.startswith(";;#ASMEND"):
            inasm = False; continue
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        if inasm and op == "buffer_load_dwordx4":
            pending.append((regs(t.split()[1].rstrip(",")), i)); nload += 1; continue
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
print("BAD" if bad else "OK")
sys.exit(1 if bad else 0)
