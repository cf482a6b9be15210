"""Compressed schedule of one kernel in a hipcc -S listing (M mfma, d dpp, r/w LDS read/write,
g/G global load/store, . waitcnt, | barrier, B branch, v other VALU): python tools/isa_sched.py FILE.s SUBSTR"""
import re
import sys

s = open(sys.argv[1]).read()
names = re.findall(r'^(_Z\S*):\s*;', s, re.M)
name = next(n for n in names if sys.argv[2] in n)
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
out = []
for l in (x.strip() for x in s[i:j].split('\n')):
    if l.startswith('.LBB'):
        out.append('\n' + l.split(':')[0] + ': ')
    elif l.startswith('v_mfma'):
        out.append('M')
    elif 'dpp' in l and l.startswith('v_'):
        out.append('d')
    elif l.startswith('ds_read'):
        out.append('r')
    elif l.startswith('ds_write'):
        out.append('w')
    elif l.startswith('s_barrier'):
        out.append('|')
    elif l.startswith(('s_cbranch', 's_branch')):
        out.append('B')
    elif l.startswith('global_load'):
        out.append('g')
    elif l.startswith('global_store'):
        out.append('G')
    elif l.startswith('s_waitcnt'):
        out.append('.')
    elif l.startswith('v_'):
        out.append('v')
print(''.join(out))
