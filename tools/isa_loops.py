"""Instruction counts of a kernel's hot loop in hipcc -S listings (A/B of code changes without a GPU):
python tools/isa_loops.py KERNEL_SUBSTRING {dpp|mfma} a.s [b.s ...]
dpp: the longest loop holding DPP row rotations (the row-layout compute chains); mfma: the longest loop holding
MFMAs. Prints total / VALU / DPP / MFMA / LDS instructions per loop body."""
import re
import sys
from collections import Counter


def loop(path, key, kind):
    s = open(path).read()
    names = re.findall(r'^(_Z\S*):\s*;', s, re.M)
    name = next(n for n in names if key in n)
    i = s.index(name + ':')
    j = s.index('.Lfunc_end', i)
    body = [l.strip().split(';')[0].strip() for l in s[i:j].split('\n')]
    body = [l for l in body if l and (not l.startswith(('.', '_Z')) or l.startswith('.LBB'))]
    lab, best = {}, None
    for k, l in enumerate(body):
        if l.endswith(':'):
            lab[l[:-1]] = k
        m = re.match(r's_cbranch_\w+\s+(\S+)|s_branch\s+(\S+)', l)
        if m:
            t = m.group(1) or m.group(2)
            if t in lab and lab[t] < k:
                seg = body[lab[t]:k + 1]
                hit = sum(1 for x in seg if ('row_ror' in x if kind == 'dpp' else 'mfma' in x))
                if hit > 20 and (best is None or len(seg) > len(best)):
                    best = seg
    return Counter(l.split()[0] + ('.dpp' if 'row_ror' in l else '') for l in best if not l.endswith(':'))


if __name__ == "__main__":
    key, kind = sys.argv[1], sys.argv[2]
    for p in sys.argv[3:]:
        c = loop(p, key, kind)
        tot = sum(c.values())
        valu = sum(v for k, v in c.items() if k.startswith('v_') and 'mfma' not in k)
        dpp = sum(v for k, v in c.items() if k.endswith('.dpp'))
        mf = sum(v for k, v in c.items() if 'mfma' in k)
        lds = sum(v for k, v in c.items() if k.startswith('ds_'))
        print(f"{p}: {tot} instructions, VALU {valu} (DPP {dpp}), MFMA {mf}, LDS {lds}")
