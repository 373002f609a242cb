"""Static instruction mix of one kernel in a hipcc -S output: straight-line code before the first loop,
inside loops (by the assembler's loop annotations), and after the last loop."""
import re, sys
s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.index(name + ":"); j = s.index(".Lfunc_end", i)
lines = [l.strip() for l in s[i:j].split("\n")]
sect, cur, seen_loop = {"prologue": [], "loop": [], "epilogue": []}, "prologue", False
for l in lines:
    if l.startswith(".LBB"):
        inloop = ("Loop Header" in l) or ("in Loop" in l) or ("Parent Loop" in l)
        if inloop: cur = "loop"; seen_loop = True
        else: cur = "epilogue" if seen_loop else "prologue"
        continue
    sect[cur].append(l)
def mix(ls):
    c = {}
    for t in ls:
        if not t or t.startswith((";", ".")): continue
        op = t.split()[0]
        k = ("mfma" if "mfma" in op else "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_"))
             else "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else None)
        if k: c[k] = c.get(k, 0) + 1
    return c
for k in sect: print(f"{k:9s}", mix(sect[k]))
