"""HBM traffic per launch of the timed render kernel from two rocprofv3 --pmc
passes (FETCH_SIZE and WRITE_SIZE cannot share a pass: 3 + 2 TCC counters > 4).

  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR WORKLOAD KERNEL_SUBSTR SAMPLES_PER_LAUNCH OUT.json

Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): rocprofv3 reports both in KiB;
on gfx950 FETCH_SIZE counts 64 B per 128-B request, so it is doubled;
WRITE_SIZE is taken as is. Infinity-Cache hits are counted by these memory-side
counters (not excluded). The summary is stamped with the kernel build hash
(bdpt_amd.kernel_build_hash) so bench.py only uses it for the same kernel."""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "bidirectional-path-tracing_amd"))
import bdpt_amd  # noqa: E402


def per_dispatch(d, counter, kernel):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter and kernel in row["Kernel_Name"]:
                vals.append(float(row["Counter_Value"]))
    return vals


fdir, wdir, workload, kernel, samples, out = sys.argv[1:7]
fetch = per_dispatch(fdir, "FETCH_SIZE", kernel)
write = per_dispatch(wdir, "WRITE_SIZE", kernel)
if not fetch or not write:
    sys.exit(f"no {kernel} dispatches with FETCH_SIZE/WRITE_SIZE under {fdir} / {wdir}")
f_kib = sum(fetch) / len(fetch)
w_kib = sum(write) / len(write)
res = {
    "config": workload,
    "kernel": kernel,
    "kernel_build": bdpt_amd.kernel_build_hash(),
    "samples_per_launch": int(samples),
    "dispatches": {"fetch_pass": len(fetch), "write_pass": len(write)},
    "fetch_size_kib_raw": f_kib,
    "write_size_kib": w_kib,
    "fetch_bytes_corrected": 2 * f_kib * 1024,
    "write_bytes": w_kib * 1024,
    "hbm_bytes_per_launch": 2 * f_kib * 1024 + w_kib * 1024,
    "correction": "FETCH_SIZE x2 (gfx950 tallies 128-B requests at 64 B); KiB -> bytes",
    "source": os.path.relpath(out, REPO),
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
