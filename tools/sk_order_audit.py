"""Audit the split-K hand-off of conv_kernel (csrc/conv.hip, small-plan 128-wide tiles) in a hipcc -S listing.

The splits of a tile publish fp32 partials and the last one to increment the tile's counter reduces them. The code
relies on relaxed agent-scope atomics (no fences, which measured slower than not splitting), so its ordering comes from
the gfx950 lowering, checked here per kernel that contains the counter increment (`global_atomic_add`):
  * every single-dword global store (the partial stores and the counter re-arm) carries `sc1` (agent-scope: written
    through past the XCD's non-coherent L2, MI355X_MICROARCH.md "Inter-workgroup visibility");
  * between the last partial store and the increment, `s_waitcnt vmcnt(0)` (the stores completed) and `s_barrier`
    (every wave's) appear, in that order;
  * after the increment, every single-dword global load (the other splits' partials) carries `sc1`, and there is
    at least one.
A toolchain change in atomic lowering or vmcnt accounting fails this CPU check instead of corrupting sums silently.
Usage: sk_order_audit.py file.s -> one line per kernel, "OK" last when all pass (exit 0), else exit 1."""
import re
import sys


def functions(lines):
    cur, body = None, []
    for ln in lines:
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur:
            if ln.startswith(".Lfunc_end"):
                yield cur, body
                cur, body = None, []
            else:
                body.append(ln.strip())
    if cur:
        yield cur, body


def audit(name, body):
    errs = []
    ia = [i for i, ln in enumerate(body) if ln.startswith("global_atomic_add ")]
    if len(ia) != 1:
        return [f"expected one counter increment, found {len(ia)}"]
    a = ia[0]
    st = [i for i, ln in enumerate(body) if re.match(r"global_store_dword\s", ln)]
    pre = [i for i in st if i < a]
    if not pre:
        errs.append("no partial store before the increment")
    for i in st:
        if not re.search(r"\bsc1\b", body[i]):
            errs.append(f"store without sc1: {body[i]}")
    if pre:
        seg = body[pre[-1] + 1:a]
        w = [k for k, ln in enumerate(seg) if re.match(r"s_waitcnt\s+vmcnt\(0\)", ln)]
        b = [k for k, ln in enumerate(seg) if ln.startswith("s_barrier")]
        if not w or not b or w[0] > b[-1]:
            errs.append("no s_waitcnt vmcnt(0) followed by s_barrier between the partial stores and the increment")
    ld = [i for i, ln in enumerate(body) if i > a and re.match(r"global_load_dword\s", ln)]
    if not ld:
        errs.append("no partial load after the increment")
    for i in ld:
        if not re.search(r"\bsc1\b", body[i]):
            errs.append(f"partial load without sc1: {body[i]}")
    return errs


def main(path):
    lines = open(path).read().splitlines()
    n, bad = 0, False
    for name, body in functions(lines):
        if not any(ln.startswith("global_atomic_add ") for ln in body):
            continue
        n += 1
        errs = audit(name, body)
        print(f"{name}: {'BAD ' + '; '.join(errs[:4]) if errs else 'ok'}")
        bad |= bool(errs)
    if n == 0:
        print("no split-K kernel found")
        return 1
    print(f"{n} split-K kernels audited")
    if bad:
        return 1
    print("OK")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
