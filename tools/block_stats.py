"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (the largest blocks):
python tools/block_stats.py <file.s> <kernel-substring> [nblocks]"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
name = sys.argv[2]
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 4
start = next(i for i, l in enumerate(lines) if l.startswith('_Z') and name in l.split(':')[0])
end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
blocks, cur = [], None
for l in lines[start:end]:
    if re.match(r'^\.LBB\d+_\d+:', l):
        cur = [l.split(':')[0], collections.Counter()]
        blocks.append(cur)
        continue
    s = l.strip()
    if l.startswith('\t') and s and not s.startswith(('.', ';')) and cur:
        cur[1][s.split()[0]] += 1
for b, c in sorted(blocks, key=lambda b: -sum(b[1].values()))[:nb]:
    f64 = sum(v for k, v in c.items() if 'f64' in k)
    ds = sum(v for k, v in c.items() if k.startswith('ds_'))
    vo = sum(v for k, v in c.items() if k.startswith('v_') and 'f64' not in k)
    print(f"{b}: {sum(c.values())} instr, f64 {f64}, ds {ds}, v_other {vo}, s_waitcnt {c['s_waitcnt']}, "
          f"s_barrier {c['s_barrier']}, scratch {sum(v for k, v in c.items() if 'scratch' in k)}")
