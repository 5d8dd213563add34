"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output (one line per kernel)."""
import re
import sys

txt = open(sys.argv[1]).read()
blocks = re.split(r"remark: [^\n]*Function Name: ", txt)
keys = [("VGPR", r"VGPRs"), ("AGPR", r"AGPRs"), ("scratch", r"ScratchSize \[bytes/lane\]"),
        ("occ", r"Occupancy \[waves/SIMD\]"), ("sgpr_spill", r"SGPRs Spill"), ("vgpr_spill", r"VGPRs Spill"),
        ("lds", r"LDS Size \[bytes/block\]")]
for b in blocks[1:]:
    name = b.split()[0]
    vals = []
    for k, pat in keys:
        m = re.search(pat + r": (\d+)", b)
        vals.append(f"{k}={m.group(1) if m else '?'}")
    print(f"{name[:58]:58s} " + " ".join(vals))
