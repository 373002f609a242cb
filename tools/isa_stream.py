"""Compact instruction stream of one kernel's MFMA region from a hipcc -S file:
M mfma, r ds_read, W ds_write, L buffer/global load, S store, p permlane, B s_barrier, . other VALU, , SALU, [..] waits.
usage: python tools/isa_stream.py <file.s> <mangled-name-substring> [max-chars]"""
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2]
i = s.index(key)
i = s.rindex('\n', 0, s.index(':', i)) + 1
name = s[i:s.index(':', i)]
j = s.index('.Lfunc_end', i)
body = [l.strip() for l in s[i:j].split('\n') if l.strip() and not l.strip().startswith(';')]
mf = [n for n, l in enumerate(body) if l.startswith('v_mfma')]
out = []
for l in body[mf[0] - 20:mf[-1] + 5]:
    op = l.split()[0]
    if op.startswith('v_mfma'): out.append('M')
    elif op.startswith('ds_read'): out.append('r')
    elif op.startswith('ds_write'): out.append('W')
    elif op.startswith(('buffer_load', 'global_load')): out.append('L')
    elif op.startswith(('buffer_store', 'global_store')): out.append('S')
    elif op.startswith('v_permlane'): out.append('p')
    elif op == 's_waitcnt': out.append('[' + l.split(None, 1)[1].replace('vmcnt', 'vm').replace('lgkmcnt', 'lgk') + ']')
    elif op == 's_barrier': out.append('B')
    elif op.startswith('v_'): out.append('.')
    elif op.startswith(('s_cbranch', 's_branch')): out.append('J')
    elif op.startswith('.LBB'): out.append('|')
    else: out.append(',')
txt = ''.join(out)
print(name, len(mf), 'MFMAs')
print(txt[:int(sys.argv[3]) if len(sys.argv) > 3 else 6000])
