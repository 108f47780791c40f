"""Sums rocprofv3 PMC counter CSVs per kernel name: python tools/pmc_summary.py DIR..."""
import csv
import glob
import os
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
            tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
            tot[k]["_dispatches"] += 0
for k, v in tot.items():
    print(k)
    for c in sorted(v):
        print(f"   {c:24s} {v[c]:.4g}")
