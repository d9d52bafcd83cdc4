"""Static instruction mix of one kernel in a hipcc -S listing: python tools/isa_mix.py k.s <name-substring>"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2]
start = name = None
for i, l in enumerate(lines):
    if re.match(r'^_Z\w*' + pat + r'\w*:', l):
        start, name = i, l
if start is None:
    sys.exit('kernel not found')
end = start
while 's_endpgm' not in lines[end]:
    end += 1
c = collections.Counter()
n = 0
for l in lines[start:end]:
    t = l.strip()
    if not t or t.startswith(('.', ';')) or t.endswith(':'):
        continue
    c[t.split()[0]] += 1
    n += 1
print(name, 'total instr', n)
for op, k in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 45):
    print(f'{k:6d} {op}')
