"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KB units) into per-launch HBM bytes.
gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports half the bytes of wide
coalesced streaming reads, so read bytes = 2 x FETCH_SIZE x 1024. Usage:
    python tools/pmc_summary.py gpurun_out/<tag> <messages_per_launch> > profiles/pmc_latest.json
"""
import csv
import json
import os
import sys

d, msgs = sys.argv[1], int(sys.argv[2])
agg = {}
for sub, ctr in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
    with open(os.path.join(d, sub, "pmc_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != ctr:
                continue
            k = r["Kernel_Name"]
            e = agg.setdefault(k, {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0, "launches": 0})
            e[ctr] += float(r["Counter_Value"])
            if ctr == "FETCH_SIZE":
                e["launches"] += 1
kt = {}
with open(os.path.join(d, "kt", "kt_kernel_stats.csv")) as f:
    for r in csv.DictReader(f):
        kt[r["Name"]] = float(r["AverageNs"])
out = {"source": d, "messages_per_launch": msgs, "kernels": {}}
for k, e in agg.items():
    n = max(e["launches"], 1)
    rd = 2 * e["FETCH_SIZE"] * 1024 / n
    wr = e["WRITE_SIZE"] * 1024 / n
    out["kernels"][k] = {"read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                         "hbm_bytes_per_launch": rd + wr, "avg_ns": kt.get(k),
                         "GBps": (rd + wr) / kt[k] if kt.get(k) else None}
dom = max((k for k in out["kernels"] if kt.get(k)), key=lambda k: kt[k])
out["kernel"] = dom
out["hbm_bytes_per_launch"] = out["kernels"][dom]["hbm_bytes_per_launch"]
print(json.dumps(out, indent=1))
