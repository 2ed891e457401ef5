"""Per-kernel instruction census of a hipcc -S output (gfx950)."""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
names = re.findall(r'^(_ZN2aa\w+):', s, re.M)
keys = ('v_mfma', 's_waitcnt', 'global_load', 'global_store', 'ds_read', 'ds_write', 's_barrier', 's_cbranch', 'buffer_', 'scratch')
for n in names:
    if len(sys.argv) > 2 and not any(k in n for k in sys.argv[2:]):
        continue
    start = s.index(n + ':')
    end = s.index('.Lfunc_end', start)
    ins = [l.strip() for l in s[start:end].split('\n')]
    ins = [l for l in ins if l and not l.startswith(('.', ';', '_'))]
    c = Counter(l.split()[0] for l in ins)
    agg = Counter()
    for k, v in c.items():
        for key in keys:
            if k.startswith(key):
                agg[key] += v
    print(n[:40], len(ins), dict(agg))
