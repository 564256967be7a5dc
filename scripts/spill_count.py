"""Spill / scalar-load counts of one kernel in a device .s file (diagnostic):
python scripts/spill_count.py file.s <kernel-symbol-substring>"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
i = next(n for n, l in enumerate(lines) if l.startswith('_ZN') and key in l.split(':')[0] and l.split(':')[0].endswith('E'))
k = i
while not lines[k].startswith('.Lfunc_end'):
    k += 1
c = collections.Counter()
for l in lines[i:k]:
    s = l.strip()
    if not s or s.startswith((';', '.')) or s.endswith(':'):
        continue
    op = s.split()[0]
    if op in ('v_writelane_b32', 'v_readlane_b32', 'v_readfirstlane_b32') or op.startswith('s_load') or op.startswith('scratch_'):
        c[op] += 1
    c['total'] += 1
# SGPR spills: writelane into a VGPR used as a spill slot (lane index immediate)
print(lines[i].split(':')[0][:60], dict(c))
