#!/usr/bin/env python3
"""Static instruction counts per source line of one kernel in a
-gline-tables-only device assembly (hipcc --cuda-device-only -S):
    python tools/asm_lines.py /tmp/idxg.s k_decode_idx [top]
Prints (file:line, total, valu, salu, lds, vmem, branch) sorted by total."""
import re, sys, collections
path, kname = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 60
files = {}
cnt = collections.defaultdict(lambda: collections.Counter())
inside = False
cur = None
for ln in open(path):
    m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', ln)
    if m:
        files[m.group(1)] = m.group(2)
        continue
    if re.match(r'^_Z\w*%s\w*:' % kname, ln) and 'Begin' not in ln:
        inside = True
        continue
    if inside and ln.startswith('.Lfunc_end'):
        break
    if not inside:
        continue
    m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', ln)
    if m:
        cur = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
        continue
    s = ln.strip()
    if not s or s.startswith(('.', ';')) or s.endswith(':'):
        continue
    op = s.split()[0]
    c = cnt[cur]
    c['all'] += 1
    if op.startswith('v_'): c['valu'] += 1
    elif op.startswith('s_cbranch') or op.startswith('s_branch'): c['br'] += 1
    elif op.startswith('s_'): c['salu'] += 1
    elif op.startswith('ds_'): c['lds'] += 1
    elif op.startswith(('global_', 'buffer_', 'flat_')): c['vmem'] += 1
tot = collections.Counter()
for c in cnt.values():
    tot.update(c)
print('total', dict(tot))
for k, c in sorted(cnt.items(), key=lambda kv: -kv[1]['all'])[:top]:
    print(f"{k:28s} {c['all']:6d} v{c['valu']:5d} s{c['salu']:5d} lds{c['lds']:4d} vm{c['vmem']:4d} br{c['br']:4d}")
