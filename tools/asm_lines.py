"""Static instruction counts per source line inside one kernel's hottest loop
(asm built with -gline-tables-only).  usage: asm_lines.py <file.s> <kernel symbol substring> [top]"""
import collections
import re
import sys

t = open(sys.argv[1]).read()
files = {m.group(1): (m.group(3) or m.group(2)).split('/')[-1]
         for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', t, re.M)}
name = next(n for n in re.findall(r'^(_Z\w+):', t, re.M) if sys.argv[2] in n)
body = t[t.index(name + ':'):t.index('.Lfunc_end', t.index(name + ':'))].split('\n')
# the depth-1 loop with the most blocks
hdrs = collections.Counter(m.group(1) for l in body for m in [re.search(r'Loop: Header=(\w+) Depth=1', l)] if m)
hdr = hdrs.most_common(1)[0][0]
cur, inloop = None, False
cnt, cntv, kinds = collections.Counter(), collections.Counter(), collections.Counter()
for l in body:
    m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', l)
    if m:
        cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
        continue
    st = l.strip()
    if re.match(r'^(\.LBB\w+:|; %bb\.\d+:)', st):  # a block starts: is it in the loop (or nested in it)?
        inloop = (f'Header={hdr} ' in l) or (f'Loop {hdr} ' in l) or bool(re.search(r'Depth=[2-9]', l)) \
            or st.startswith('.L' + hdr + ':')
        continue
    s = l.strip()
    if not inloop or not s or s.startswith(('.', ';')):
        continue
    op = s.split()[0]
    cnt[cur] += 1
    kinds[op.split('_')[0]] += 1
    if op.startswith('v_'):
        cntv[cur] += 1
print('loop', hdr, 'instructions', sum(cnt.values()), dict(kinds.most_common(8)))
for k, v in cntv.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    print(f'{k[0]}:{k[1]}  valu {v}  all {cnt[k]}')
