"""Per-kernel table of rocprofv3 PMC counters (sums over dispatches) from counters.sh output."""
import csv
import glob
import sys

d = sys.argv[1]
agg = {}
for f in sorted(glob.glob(f"{d}/pmc*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if k.startswith("__amd") or k in ("scale_even_rows_kernel", "key_to_ntt_kernel"):
            continue
        agg.setdefault(k, {})
        agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k, c in agg.items():
    print(k)
    for n, v in sorted(c.items()):
        print(f"   {n:28s} {v:16.4g}")
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
        wc = c["SQ_WAVE_CYCLES"]
        for n in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if n in c:
                print(f"   {n + '/WAVE_CYCLES':40s} {c[n] / wc:.3f}")
    if "TCC_HIT_sum" in c:
        print(f"   L2 hit rate {c['TCC_HIT_sum'] / max(1, c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.3f}")
