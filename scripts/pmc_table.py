#!/usr/bin/env python3
"""Per-kernel sums of every counter found in rocprofv3 --pmc output directories."""
import csv
import glob
import os
import sys
from collections import defaultdict

tab = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?").split("(")[0]
            tab[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add((d, r.get("Dispatch_Id")))
names = sorted({c for k in tab for c in tab[k]})
for k in sorted(tab, key=lambda k: -tab[k].get("SQ_WAVE_CYCLES", 0)):
    print(k[:40], " ".join(f"{c}={tab[k][c]:.4g}" for c in names if c in tab[k]))
