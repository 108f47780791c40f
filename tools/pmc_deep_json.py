"""Issue / latency counters of the timed render kernel, per launch, from the
rocprofv3 --pmc passes of tools/profile_round.sh (one pass per counter group).

  python tools/pmc_deep_json.py DIR WORKLOAD KERNEL_SUBSTR SAMPLES_PER_LAUNCH CUS OUT.json [XCDS=8]

Derived (MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_*
count quad-cycles; a wave64 VALU instruction issues over 2 cycles;
GRBM_GUI_ACTIVE is summed over the XCDs — 8.8e9 for a 464 ms launch at
~2.4 GHz = 8 x 1.1e9):
  active_lane_frac = SQ_THREAD_CYCLES_VALU / (64 * SQ_INSTS_VALU)
                     (lanes enabled per VALU instruction, averaged)
  valu_issue_frac  = 2 * SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / XCDS * CUS * 4 SIMDs)
                     (SIMD cycles spent issuing VALU over the SIMDs' cycles)
  valu_lane_util   = valu_issue_frac * active_lane_frac (useful fraction of VALU lane-cycles)
  wait_frac        = SQ_WAIT_ANY / SQ_WAVE_CYCLES (wave cycles waiting on anything)
Stamped with the kernel build hash (bdpt_amd.kernel_build_hash)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "bidirectional-path-tracing_amd"))
import bdpt_amd  # noqa: E402

d, workload, kernel, samples, cus, out = sys.argv[1:7]
samples, cus = int(samples), int(cus)
xcds = int(sys.argv[7]) if len(sys.argv) > 7 else 8
vals = defaultdict(list)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if kernel in row["Kernel_Name"]:
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
if not vals:
    sys.exit(f"no {kernel} dispatches under {d}")
c = {k: sum(v) / len(v) for k, v in vals.items()}  # per launch
res = {"config": workload, "kernel": kernel, "kernel_build": bdpt_amd.kernel_build_hash(),
       "samples_per_launch": samples, "cus": cus, "counters_per_launch": c}


def g(k):
    return c.get(k)


if g("SQ_THREAD_CYCLES_VALU") and g("SQ_INSTS_VALU"):
    res["active_lane_frac"] = round(g("SQ_THREAD_CYCLES_VALU") / (64 * g("SQ_INSTS_VALU")), 4)
if g("SQ_INSTS_VALU") and g("GRBM_GUI_ACTIVE"):
    res["valu_issue_frac"] = round(2 * g("SQ_INSTS_VALU") / (g("GRBM_GUI_ACTIVE") / xcds * cus * 4), 4)
if "active_lane_frac" in res and "valu_issue_frac" in res:
    res["valu_lane_util"] = round(res["active_lane_frac"] * res["valu_issue_frac"], 4)
if g("SQ_WAIT_ANY") and g("SQ_WAVE_CYCLES"):
    res["wait_frac"] = round(g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"), 4)
if g("SQ_INSTS_VALU"):
    res["valu_insts_per_sample"] = round(g("SQ_INSTS_VALU") / samples, 1)
if g("SQ_INSTS_SALU"):
    res["salu_insts_per_sample"] = round(g("SQ_INSTS_SALU") / samples, 1)
if g("SQ_INSTS_VMEM_RD"):
    res["vmem_rd_insts_per_sample"] = round(g("SQ_INSTS_VMEM_RD") / samples, 2)
if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum"):
    res["l2_hit_rate"] = round(g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")), 4)
# the kernel's limiter: VALU issue at low lane utilisation when the SIMDs spend a large
# share of their cycles issuing VALU with few lanes enabled; latency when waves mostly wait
vi, al, wf = res.get("valu_issue_frac", 0), res.get("active_lane_frac", 1), res.get("wait_frac", 0)
res["limiter"] = ("VALU issue at low lane utilisation (divergence)" if vi >= 0.3 and al < 0.5
                  else "latency" if wf >= 0.5 else "issue" if vi >= 0.5 else "undetermined")
res["source"] = os.path.relpath(out, REPO)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "counters_per_launch"}))
