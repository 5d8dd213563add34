"""Per-step ISA census of a kernel's CMUX step loop from a hipcc -S listing.

    python tools/isa_census.py <context.s> <kernel> <block>=<count> [<block>=<count> ...] [--json out]

Each <block> is a basic-block label of the kernel (e.g. .LBB2_17) and <count> how many times one CMUX
step executes it (from the loop structure: tools/block_stats.py lists the blocks). The census sums
every instruction of those blocks x count into buckets, so the result is the static instruction
stream of one step of one wave. Cross-check: the FP64 and VALU totals per step must agree with the
SQ_INSTS_VALU_*_F64 / SQ_INSTS_VALU counters per message / (rotations x steps x 64 lanes).
"""
import collections
import json
import re
import sys

BUCKETS = [
    ("fp64 add/mul/fma", lambda o: o.startswith(("v_add_f64", "v_mul_f64", "v_fma_f64", "v_fmac_f64"))),
    ("fp64 other (cvt, floor, rndne, ldexp)", lambda o: o.startswith("v_") and "f64" in o),
    ("permlane (relayouts)", lambda o: "permlane" in o),
    ("bit-field extract", lambda o: o.startswith(("v_bfe_", "v_alignbit"))),
    ("int add/sub", lambda o: re.match(r"v_(add|sub|subrev)(3)?_(u|i|co_u|nc_u)32", o) is not None),
    ("int min/max/logic", lambda o: re.match(r"v_(min|max|min3|max3|and|or|xor|and_or|or3|xad|lshl_or|lshl_add|"
                                                r"add_lshl|bfi|cndmask)", o) is not None),
    ("int shift", lambda o: re.match(r"v_(lshl|lshr|ashr)", o) is not None),
    ("v_mov / readfirstlane", lambda o: o.startswith(("v_mov", "v_readfirstlane", "v_readlane", "v_writelane"))),
    ("other VALU", lambda o: o.startswith("v_")),
    ("LDS read", lambda o: o.startswith("ds_read")),
    ("LDS write", lambda o: o.startswith("ds_write")),
    ("other LDS", lambda o: o.startswith("ds_")),
    ("VMEM (incl. LDS-DMA)", lambda o: o.startswith(("buffer_", "global_", "flat_"))),
    ("s_waitcnt", lambda o: o == "s_waitcnt"),
    ("s_barrier", lambda o: o == "s_barrier"),
    ("SALU / branch / other", lambda o: True),
]


def blocks(path, kernel):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and kernel in l.split(":")[0]
                 and "guard" not in l.split(":")[0])
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    out, cur = collections.OrderedDict(), "entry"
    out[cur] = collections.Counter()
    for l in lines[start:end]:
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            cur = m.group(1)
            out[cur] = collections.Counter()
            continue
        s = l.strip()
        if l.startswith("\t") and s and not s.startswith((".", ";")):
            op = s.split()[0]
            out[cur][op] += 1
            if op.startswith("v_") and "f64" in op and "s[" in s:  # FP64 op reading an SGPR pair
                out[cur]["@sgpr:" + op] += 1
            if op.startswith("s_cbranch"):  # the fall-through code is a block of its own: <label>+<k>
                base = cur.split("+")[0]
                k = int(cur.split("+")[1]) + 1 if "+" in cur else 1
                cur = f"{base}+{k}"
                out[cur] = collections.Counter()
    return out


def census(path, kernel, counts):
    bl = blocks(path, kernel)
    tot = collections.Counter()
    for b, n in counts.items():
        for op, c in bl[b].items():
            tot[op] += c * n
    res = collections.OrderedDict((name, 0) for name, _ in BUCKETS)
    for op, c in tot.items():
        if op.startswith("@"):
            continue
        for name, f in BUCKETS:
            if f(op):
                res[name] += c
                break
    valu = sum(c for op, c in tot.items() if op.startswith("v_"))
    res["fp64 with an SGPR operand (of the above)"] = sum(c for op, c in tot.items() if op.startswith("@sgpr:"))
    return res, valu, tot


def list_blocks(path, kernel):
    for b, c in blocks(path, kernel).items():
        v = sum(n for o, n in c.items() if o.startswith("v_"))
        f = sum(n for o, n in c.items() if o.startswith(("v_add_f64", "v_mul_f64", "v_fma_f64", "v_fmac_f64")))
        br = [o for o in c if o.startswith(("s_cbranch", "s_branch"))]
        print(f"{b:14s} instr {sum(n for o, n in c.items() if not o.startswith('@')):5d} valu {v:5d} fp64 {f:5d} lds {sum(n for o, n in c.items() if o.startswith('ds_')):4d} {br}")


if __name__ == "__main__":
    if len(sys.argv) == 3:
        list_blocks(sys.argv[1], sys.argv[2])
        sys.exit(0)
    args = [a for a in sys.argv[1:] if not a.startswith("--json")]
    jpath = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--json=")), None)
    path, kernel = args[0], args[1]
    counts = {a.split("=")[0]: float(a.split("=")[1]) for a in args[2:]}
    res, valu, tot = census(path, kernel, counts)
    fp64 = res["fp64 add/mul/fma"]
    print(f"{kernel}: one CMUX step of one wave ({', '.join(f'{b} x{n:g}' for b, n in counts.items())})")
    print(f"  VALU {valu:.0f} (fp64 add/mul/fma {fp64:.0f} = {fp64 / valu:.1%}; non-fp64 {valu - fp64:.0f} = "
          f"{(valu - fp64) / valu:.1%})")
    for name, c in res.items():
        share = f"{c / valu:6.1%} of VALU" if name in [n for n, _ in BUCKETS[:9]] else ""
        print(f"  {name:40s} {c:7.0f}  {share}")
    if jpath:
        json.dump({"kernel": kernel, "blocks": counts, "valu": valu, "buckets": res,
                   "opcodes": dict(sorted(tot.items(), key=lambda kv: -kv[1]))}, open(jpath, "w"), indent=1)
