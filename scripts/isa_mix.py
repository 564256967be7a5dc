"""Static instruction mix of one kernel in a device .s file (diagnostic):
python scripts/isa_mix.py file.s <kernel-symbol-substring> [start-marker end-marker]"""
import collections
import sys

lines = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
i = next(n for n, l in enumerate(lines) if l.startswith('_ZN') and key in l.split(':')[0] and l.split(':')[0].endswith('E'))
k = i
while not lines[k].startswith('.Lfunc_end'):
    k += 1
body = lines[i:k]
c = collections.Counter()
ops = collections.Counter()
for l in body:
    l = l.strip()
    if not l or l.startswith(';') or l.startswith('.') or l.endswith(':'):
        continue
    op = l.split()[0]
    cls = ('valu' if op.startswith('v_') else 'salu' if op.startswith('s_') else 'ds' if op.startswith('ds_')
           else 'vmem' if op.startswith(('global_', 'buffer_', 'flat_', 'scratch_')) else 'other')
    c[cls] += 1
    ops[op] += 1
print(lines[i].split(':')[0], 'static lines', len(body))
print(dict(c))
print(ops.most_common(40))
