"""Instruction mix of one kernel in a hipcc -S listing: python tools/isa_mix.py FILE.s SUBSTRING [loop]
(`loop`: only the body of the kernel's longest basic-block loop, i.e. between the label with the most
instructions before its back-branch)."""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
names = re.findall(r'^(_Z\S*):\s*;', s, re.M)
name = next(n for n in names if sys.argv[2] in n)
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
body = s[i:j].split('\n')
ins = [l.strip().split(';')[0].strip() for l in body
       if l.strip() and (l.strip().startswith('.LBB') or not l.strip().startswith(('.', ';', '_Z')))]
if len(sys.argv) > 3:      # longest loop: label ... s_cbranch back to that label
    labels = {}
    best = (0, 0, 0)
    for k, l in enumerate(ins):
        if l.endswith(':'):
            labels[l[:-1]] = k
        m = re.match(r's_cbranch_\w+\s+(\S+)|s_branch\s+(\S+)', l)
        if m:
            t = m.group(1) or m.group(2)
            if t in labels and k - labels[t] > best[0]:
                best = (k - labels[t], labels[t], k)
    ins = ins[best[1]:best[2] + 1]
c = Counter(l.split()[0] for l in ins if not l.endswith(':'))
print(name, sum(c.values()), "instructions")
for op, n in c.most_common(60):
    print(f"{n:6d} {op}")
