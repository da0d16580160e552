"""Average per-launch value of every collected counter, per attention kernel, from
rocprofv3 --pmc output directories.  Usage: python tools/pmc_sq.py <dir> [<dir> ...]"""
import csv
import glob
import sys
from collections import defaultdict

vals = defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            short = next((s for s in ("attn_fwd", "attn_dq", "attn_dkdv4", "attn_dkdv", "attn_bwd") if s + "_kernel" in k),
                         None)
            if short:
                vals[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    print(f"{k:12s} {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
