"""Instruction statistics of one kernel in a hipcc -S listing (build/context.s):
python tools/isa_stats.py <file.s> <kernel-substring> [more files...]"""
import collections
import sys


def stats(path, name):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith('_Z') and name in l.split(':')[0])
    end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
    ins = [l.strip().split()[0] for l in lines[start:end]
           if l.startswith('\t') and l.strip() and not l.strip().startswith(('.', ';'))]
    return collections.Counter(ins)


if __name__ == "__main__":
    name = sys.argv[2]
    for p in [sys.argv[1]] + sys.argv[3:]:
        c = stats(p, name)
        tot = sum(c.values())
        grp = lambda f: sum(v for k, v in c.items() if f(k))
        print(f"{p}: {tot} instr, f64 {grp(lambda k: 'f64' in k)}, ds {grp(lambda k: k.startswith('ds_'))}, "
              f"global {grp(lambda k: k.startswith(('global_', 'buffer_')))}, scratch {grp(lambda k: 'scratch' in k)}, "
              f"s_barrier {c['s_barrier']}, s_waitcnt {c['s_waitcnt']}, v_ (non-f64) {grp(lambda k: k.startswith('v_') and 'f64' not in k)}")
