#!/usr/bin/env python3
"""Per-basic-block scratch (spill) and f64-add counts of one kernel in a hipcc -S assembly file:
   tools/isa_spills.py file.s kernel_substring"""
import re
import sys

src = open(sys.argv[1]).read()
pat = sys.argv[2]
m = [mm for mm in re.finditer(r"^(_Z\S+):", src, re.M) if pat in mm.group(1)]
if not m:
    sys.exit('kernel not found')
start = m[0].end()
end = src.find('.Lfunc_end', start)
blk, stats, order = 'entry', {}, []
for line in src[start:end].split('\n'):
    b = re.match(r'^(\.LBB\d+_\d+):(.*)$', line)
    if b:
        blk = b.group(1) + ' ' + b.group(2).strip().lstrip(';').strip()
        continue
    s = line.strip()
    if not s or s.startswith(';') or s.startswith('.'):
        continue
    if blk not in stats:
        stats[blk] = [0, 0, 0]
        order.append(blk)
    st = stats[blk]
    st[0] += 1
    if 'scratch_' in s:
        st[1] += 1
    if s.startswith('v_add_f64'):
        st[2] += 1
tot = [0, 0, 0]
for b in order:
    st = stats[b]
    for k in range(3):
        tot[k] += st[k]
    if st[1] or st[2] >= 8:
        print(f'{b[:70]:70s} insts {st[0]:5d} scratch {st[1]:4d} add_f64 {st[2]:3d}')
print('total', tot)

# optional 3rd argument: a basic-block label (e.g. .LBB4_96) -> instruction histogram of that block
if len(sys.argv) > 3:
    want = sys.argv[3]
    body = src[start:end].split('\n')
    on, hist = False, {}
    for line in body:
        b = re.match(r'^(\.LBB\d+_\d+):', line)
        if b:
            on = b.group(1) == want
            continue
        s = line.strip()
        if on and s and not s.startswith(';') and not s.startswith('.'):
            op = s.split()[0]
            hist[op] = hist.get(op, 0) + 1
    for op, c in sorted(hist.items(), key=lambda kv: -kv[1])[:30]:
        print(f'{c:5d} {op}')
