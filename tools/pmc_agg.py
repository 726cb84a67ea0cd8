"""Average rocprofv3 --pmc counter values per launch for kernels matching a name.

    python tools/pmc_agg.py <counter_collection.csv> <kernel-substring>
"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
agg: dict = {}
for r in rows:
    agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} n={len(v):3d} mean={sum(v) / len(v):.6g}")
