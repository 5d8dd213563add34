"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KB units) into per-launch HBM bytes.
gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports half the bytes of wide
coalesced streaming reads, so read bytes = 2 x FETCH_SIZE x 1024; with a pmc_l2 pass, the L1 -> L2
read bytes (TCP_TCC_READ_REQ_sum x 128 B) and the L2 hit rate per kernel. Usage:
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
# L1 -> L2 read requests (128 B each: a 16 B-per-lane wave load is 8 of them) and L2 hits / misses,
# when the round profile ran that pass (pmc_l2)
l2f = os.path.join(d, "pmc_l2", "pmc_counter_collection.csv")
if os.path.exists(l2f):
    l2, disp = {}, {}
    with open(l2f) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"]
            l2.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
            l2[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp.setdefault(k, set()).add(r["Dispatch_Id"])
    for k, c in l2.items():
        if k in out["kernels"] and "TCP_TCC_READ_REQ_sum" in c:
            n = max(len(disp[k]), 1)
            out["kernels"][k]["l2_read_bytes_per_launch"] = c["TCP_TCC_READ_REQ_sum"] * 128 / n
            hm = c.get("TCC_HIT_sum", 0.0) + c.get("TCC_MISS_sum", 0.0)
            out["kernels"][k]["l2_hit_rate"] = c.get("TCC_HIT_sum", 0.0) / hm if hm else None
dom = max((k for k in out["kernels"] if kt.get(k)), key=lambda k: kt[k])
out["kernel"] = dom
out["hbm_bytes_per_launch"] = out["kernels"][dom]["hbm_bytes_per_launch"]
print(json.dumps(out, indent=1))
