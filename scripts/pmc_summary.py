"""Per-kernel mean of every PMC counter in rocprofv3 counter_collection CSVs."""
import csv
import os
import sys
from collections import defaultdict

for path in sys.argv[1:]:
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0][:70]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        if os.environ.get("PMC_FILTER", "decode") not in k:
            continue
        n = len(disp[k])
        print(path, k, "dispatches", n)
        for c in sorted(v):
            print(f"   {c:24s} {v[c] / n:16.0f}")
