"""Dump the instructions of one basic block of a kernel in a hipcc -S listing, optionally only
those whose mnemonic starts with a prefix: python tools/block_dump.py <file.s> <kernel> <label> [prefix...]"""
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
name, label = sys.argv[2], sys.argv[3]
prefixes = tuple(sys.argv[4:])
start = next(i for i, l in enumerate(lines) if l.startswith('_Z') and name in l.split(':')[0])
end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
inb = False
for l in lines[start:end]:
    if re.match(r'^\.LBB\d+_\d+:', l):
        if inb:
            break
        inb = l.split(':')[0] == label
        continue
    s = l.strip()
    if inb and l.startswith('\t') and s and not s.startswith(('.', ';')):
        if not prefixes or s.split()[0].startswith(prefixes):
            print(s)
