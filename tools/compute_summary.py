"""Per-message FP64 VALU work of the detect kernels from a tools/counters.sh run (SQ counters
are per wave instruction; x64 lanes). Usage:
    python tools/compute_summary.py gpurun_out/<tag> <messages_per_launch> > profiles/compute_latest.json
bench.py divides these counts by the live kernel time for the "compute" roofline object."""
import csv
import glob
import json
import sys

d, msgs = sys.argv[1], int(sys.argv[2])
ctrs = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
        "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU", "SQ_INSTS_LDS")
agg, launches = {}, {}
for f in sorted(glob.glob(f"{d}/pmc*/pmc_counter_collection.csv")):
    seen = set()
    for r in csv.DictReader(open(f)):
        k, c = r["Kernel_Name"], r["Counter_Name"]
        if c not in ctrs:
            continue
        agg.setdefault(k, {}).setdefault(c, 0.0)
        agg[k][c] += float(r["Counter_Value"])
        if (k, r.get("Dispatch_Id", r.get("Correlation_Id"))) not in seen and c == ctrs[0]:
            seen.add((k, r.get("Dispatch_Id", r.get("Correlation_Id"))))
            launches[k] = launches.get(k, 0) + 1
out = {"source": f"profiles/<tag>/compute_summary.json from {d}", "messages_per_launch": msgs, "lanes": 64, "kernels": {}}
for k, c in agg.items():
    if not all(x in c for x in ctrs[:4]):
        continue
    n = max(1, launches.get(k, 1))
    fp64 = sum(c[x] for x in ctrs[:4]) * 64 / n / msgs
    flops = (c[ctrs[0]] + c[ctrs[1]] + c[ctrs[3]] + 2 * c[ctrs[2]]) * 64 / n / msgs
    out["kernels"][k] = {"fp64_lane_instr_per_msg": fp64, "fp64_flop_per_msg": flops,
                         "valu_lane_instr_per_msg": c.get("SQ_INSTS_VALU", 0) * 64 / n / msgs,
                         "lds_instr_per_msg": c.get("SQ_INSTS_LDS", 0) / n / msgs}
print(json.dumps(out, indent=1))
