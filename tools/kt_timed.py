#!/usr/bin/env python3
"""Per-launch durations of the frame kernels in a rocprofv3 kernel trace, next to the
bench line that ran under it (tools/gpu_runs/run.sh final_b): the trace's stats CSV
averages every launch of a run (the in-run parity render of every 5th row, the
counting pass), so the launches the bench timed are picked out here — the last
`steps` full-frame launches before the parity render — and their mean is compared
with the line's roofline.kernel_ms (HIP events on the launch stream).

usage: kt_timed.py PROF_DIR LABEL   (PROF_DIR/kt_<config>/kt_kernel_trace.csv,
                                     gpurun_out/LABEL_bench_<config>.json)"""
import csv
import glob
import json
import os
import sys

prof, label = sys.argv[1], sys.argv[2]
for d in sorted(glob.glob(os.path.join(prof, "kt_*"))):
    cfg = os.path.basename(d)[3:]
    bench = os.path.join(os.path.dirname(prof.rstrip("/")), f"{label}_bench_{cfg}.json")
    lines = [json.loads(l) for l in open(bench) if l.startswith("{")] if os.path.exists(bench) else []
    if not lines:
        continue
    b = lines[-1]
    roof = b.get("roofline") or {}
    kname = roof.get("kernel") or ("pt_frame_kernel" if cfg.startswith(("path_", "direct_")) else "")
    rows = [r for r in csv.DictReader(open(os.path.join(d, "kt_kernel_trace.csv")))
            if kname and f"::{kname}<" in r["Kernel_Name"]]
    # the frame launches, in dispatch order, without the counting pass (template <_, true, _> of the bdpt kernels)
    rows = [r for r in rows if kname.startswith("pt_") or ", true, " not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    steps, warm = b["steps"], b["warmup"]
    timed = durs[warm:warm + steps]
    mean = sum(timed) / len(timed) if timed else float("nan")
    km = roof.get("kernel_ms", b["config"].get("kernel_ms"))
    print(f"{cfg}: {len(durs)} launches {[round(x, 2) for x in durs]}; timed (after {warm} warmup) "
          f"mean {mean:.3f} ms; bench kernel_ms {km}; ms_per_step {b['ms_per_step']}; value {b['value']} {b['unit']}")
