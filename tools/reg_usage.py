"""Print VGPR count and scratch bytes of every k_solve_reg instance from an unbundled
gfx950 code object's notes:  llvm-readelf --notes dev.co | python tools/reg_usage.py"""
import re
import sys

cur, rows = {}, []
for line in sys.stdin:
    m = re.match(r'\s*-?\s*\.(\w+):\s+(\S+)', line)
    if not m:
        continue
    k, v = m.groups()
    if k == 'agpr_count' and cur:
        rows.append(cur)
        cur = {}
    cur[k] = v
rows.append(cur)
for r in rows:
    if 'solve_reg' in r.get('name', ''):
        inst = re.findall(r'ILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E', r['name'])
        print(inst[0] if inst else r['name'], 'vgpr', r.get('vgpr_count'), 'scratch', r.get('private_segment_fixed_size'))
