"""Static instruction counts of one kernel by source function (diagnostic): compile with
-gline-tables-only -S, then
  python scripts/isa_by_source.py file.s <kernel-symbol-substring> [csrc dir]
Each instruction is attributed to the innermost source line of its .loc (inlined code keeps
its own line), lines to the enclosing function definition of that source file."""
import collections
import os
import re
import sys

asm, key = sys.argv[1], sys.argv[2]
csrc = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-td_amd", "csrc")
lines = open(asm).read().split("\n")
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
    if m:
        files[int(m.group(1))] = m.group(3)
i = next(n for n, l in enumerate(lines) if l.startswith("_ZN") and key in l.split(":")[0] and l.split(":")[0].endswith("E"))
k = i
while not lines[k].startswith(".Lfunc_end"):
    k += 1

fdefs = {}  # file -> sorted [(line, name)]
def funcs(fname):
    if fname not in fdefs:
        out = []
        p = os.path.join(csrc, fname)
        if os.path.exists(p):
            for n, t in enumerate(open(p).read().split("\n"), 1):
                m = re.match(r'\s*(?:template\s*<[^>]*>\s*)?(?:static\s+)?(?:__global__|__device__|__host__|TD_HD|struct)\b.*?(\w+)\s*\(', t)
                if m and not t.strip().endswith(";"):
                    out.append((n, m.group(1)))
                m2 = re.match(r'\s*(?:__device__|TD_HD)[^(]*\b(\w+)\s*\([^;]*\{?\s*$', t)
        fdefs[fname] = out
    return fdefs[fname]

def func_of(fname, line):
    best = "?"
    for n, name in funcs(fname):
        if n <= line:
            best = name
        else:
            break
    return "%s:%s" % (fname, best)

cur = ("?", 0)
by_func = collections.defaultdict(collections.Counter)
by_line = collections.Counter()
for l in lines[i:k]:
    s = l.strip()
    m = re.match(r'\.loc\s+(\d+)\s+(\d+)', s)
    if m:
        cur = (files.get(int(m.group(1)), "?"), int(m.group(2)))
        continue
    if not s or s.startswith((";", ".")) or s.endswith(":"):
        continue
    op = s.split()[0]
    cls = ('valu' if op.startswith('v_') else 'salu' if op.startswith('s_') else 'ds' if op.startswith('ds_')
           else 'vmem' if op.startswith(('global_', 'buffer_', 'flat_', 'scratch_')) else 'other')
    f = func_of(*cur)
    by_func[f][cls] += 1
    by_line[cur] += 1
tot = collections.Counter()
for c in by_func.values():
    tot.update(c)
print(lines[i].split(":")[0], dict(tot))
for f, c in sorted(by_func.items(), key=lambda kv: -sum(kv[1].values()))[:40]:
    print("%-45s %5d  %s" % (f, sum(c.values()), dict(c)))
print("top lines:")
for (fn, ln), n in by_line.most_common(25):
    print("  %s:%d %d" % (fn, ln, n))
