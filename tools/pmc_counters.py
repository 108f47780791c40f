"""Per-launch totals of every counter of a rocprofv3 --pmc pass for one kernel,
and per camera sample (samples_per_launch from the bench JSON line in the log).
  python tools/pmc_counters.py RAW_DIR KERNEL_SUBSTR BENCH_LOG"""
import collections
import csv
import glob
import json
import os
import sys

raw, kernel, log = sys.argv[1:4]
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(raw, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if kernel in row["Kernel_Name"]:
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
samples = None
for line in open(log):
    if line.startswith("{"):
        try:
            samples = json.loads(line)["roofline"]["samples_per_launch"]
        except (ValueError, KeyError):
            pass
out = {"kernel": kernel, "samples_per_launch": samples, "per_launch": {}, "per_sample": {}}
for k, v in sorted(vals.items()):
    out["per_launch"][k] = sum(v) / len(v)
    if samples:
        out["per_sample"][k] = round(sum(v) / len(v) / samples, 4)
out["dispatches"] = {k: len(v) for k, v in vals.items()}
print(json.dumps(out, indent=1))
