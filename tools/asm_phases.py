#!/usr/bin/env python3
"""Static instruction counts of k_decode_idx by decode_block phase (the
call-site line inside decode_block / index_block from each .loc's inline
chain) in a -gline-tables-only device assembly:
    python tools/asm_phases.py /tmp/idxg.s"""
import re, sys, collections
PH = [(487, 655, 'pass1'), (1339, 1430, 'setup'), (1431, 1476, 'stage+cut'), (1477, 1509, 'global'),
      (1510, 1529, 'starts'), (1530, 1574, 'P parse'), (1575, 1653, 'HBM loads'),
      (1654, 1697, 'literals'), (1698, 1761, 'HBM stores'), (1762, 1787, 'ring'),
      (1788, 1805, 'flush'), (1805, 1830, 'end')]
def phase(line):
    for a, b, n in PH:
        if a <= line <= b:
            return n
    return 'other:%d' % line
path = sys.argv[1]
lines = open(path).read().split('\n')
start = next(i for i, l in enumerate(lines) if re.match(r'^_ZN6lz4ada3idx12k_decode_idxE\w*:', l))
cnt = collections.defaultdict(collections.Counter)
cur = 'none'
for l in lines[start:]:
    if l.startswith('.Lfunc_end'):
        break
    m = re.match(r'\s*\.loc\s+\d+\s+\d+.*?;\s*(.*)$', l)
    if m:
        chain = re.findall(r'lz4ada_idx\.hip:(\d+)', m.group(1))
        chain = [int(x) for x in chain]
        inner = [x for x in chain if not (1837 <= x <= 1889)]
        cur = phase(inner[-1]) if inner else 'kernel'
        continue
    s = l.strip()
    if not s or s.startswith(('.', ';')) or s.endswith(':'):
        continue
    op = s.split()[0]
    c = cnt[cur]
    c['all'] += 1
    if op.startswith('v_'): c['valu'] += 1
    elif op.startswith(('s_cbranch', 's_branch')): c['br'] += 1
    elif op.startswith('s_waitcnt') or op.startswith('s_nop'): c['wait'] += 1
    elif op.startswith('s_'): c['salu'] += 1
    elif op.startswith('ds_'): c['lds'] += 1
    elif op.startswith(('global_', 'buffer_', 'flat_')): c['vmem'] += 1
for k, c in sorted(cnt.items(), key=lambda kv: -kv[1]['all']):
    print(f"{k:14s} {c['all']:6d} v{c['valu']:5d} s{c['salu']:5d} br{c['br']:4d} w{c['wait']:4d} lds{c['lds']:4d} vm{c['vmem']:4d}")
