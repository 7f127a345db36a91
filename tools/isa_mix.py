"""Static instruction mix of one kernel, per basic block, with the source lines each block
comes from (build with -gline-tables-only --save-temps).  Usage:
  python tools/isa_mix.py FILE.s KERNEL_SUBSTRING [min_block_len]"""
import collections
import re
import sys

path, sub = sys.argv[1], sys.argv[2]
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 12
L = open(path).read().split('\n')
st = [i for i, l in enumerate(L) if re.match(r'^_Z\S*:', l) and sub in l][0]
en = [i for i in range(st, len(L)) if L[i].startswith('.Lfunc_end')][0]
blocks, cur, line = [], ['entry', [], collections.Counter()], (0, 0)
for l in L[st:en]:
    m = re.match(r'^(\.LBB\S+):', l)
    if m:
        blocks.append(cur)
        cur = [m.group(1), [], collections.Counter()]
        continue
    s = l.strip()
    m = re.match(r'\.loc\s+(\d+)\s+(\d+)', s)
    if m:
        line = (int(m.group(1)), int(m.group(2)))
        continue
    if not s or s.startswith(';') or s.startswith('.'):
        continue
    cur[1].append(s.split()[0])
    cur[2][line] += 1
blocks.append(cur)
for n, ins, lines in blocks:
    if len(ins) < minlen:
        continue
    c = collections.Counter()
    for i in ins:
        k = ('pk' if i.startswith('v_pk_') else 'mfma' if i.startswith('v_mfma') else 'v' if i.startswith('v_')
             else 'ds' if i.startswith('ds_') else 'vm' if i.startswith(('global_', 'buffer_')) else 's')
        c[k] += 1
    br = [i for i in ins if i.startswith('s_cbranch')]
    top = ' '.join(f'{f}:{ln}x{k}' for (f, ln), k in sorted(lines.items(), key=lambda x: -x[1])[:6])
    print(f'{n:12s} n={len(ins):4d} ' + ' '.join(f'{k}={c[k]}' for k in ('v', 'pk', 'mfma', 'ds', 'vm', 's')) + f' | {top}')
