#!/bin/bash
# Round profile of a bench workload (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats of bench.py (kernel time per launch)
#   2. --pmc FETCH_SIZE pass, 3. --pmc WRITE_SIZE pass (separate: TCC counter budget)
#   4. issue / latency counter groups, one pass each (per-block limits of MI355X_MICROARCH.md)
#   -> gpurun_out/prof_TAG/{kernel_stats_<workload>.csv, pmc_<workload>.json, pmc_deep_<workload>.json}
#      (stamped with the kernel build hash; bench.py uses them, copied to profiles/, only for that build)
# usage: tools/profile_round.sh TAG SCENE W H SPP
set -e
cd "$(dirname "$0")/.."
TAG=$1 SCENE=${2:-caustic} W=${3:-512} H=${4:-512} SPP=${5:-256}
R=$PWD
WL=${SCENE}_${W}x${H}_${SPP}spp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu --scene $SCENE --width $W --height $H --spp $SPP"
K=${KERNEL:-"bdpt_frame_kernel<false, false, false>"}  # KERNEL=bdpt_frame_kernel_split<...> for rrDepth <= 3 scenes
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_$WL -o kt --output-format csv -- $B --steps 2 --warmup 1 > $OUT/kt_$WL.log 2>&1
# the frame-kernel build that ran (bdpt_frame_kernel, _split for rrDepth <= 3, ...), unless KERNEL names it
if [ -z "$KERNEL" ]; then
  K=$(python3 - "$(find $OUT/kt_$WL -name '*kernel_stats.csv' | head -1)" <<'PY'
import csv, re, sys
best = max((r for r in csv.DictReader(open(sys.argv[1])) if "bdpt_frame_kernel" in r["Name"]),
           key=lambda r: float(r["TotalDurationNs"]))
print(re.search(r"(bdpt_frame_kernel\w*<[^>]*>)", best["Name"]).group(1))
PY
)
fi
echo "frame kernel: $K"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch_$WL -o fetch --output-format csv -- $B --steps 1 --warmup 0 > $OUT/fetch_$WL.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write_$WL -o write --output-format csv -- $B --steps 1 --warmup 0 > $OUT/write_$WL.log 2>&1
i=0
while read -r grp; do
  i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d $OUT/deep_$WL/p$i -o p$i --output-format csv -- $B --steps 1 --warmup 0 > $OUT/deep_${WL}_p$i.log 2>&1
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU
GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum
GROUPS
cd $R
find $OUT/kt_$WL -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_$WL.csv \;
SAMPLES=$((W * H * SPP))
CUS=$(python3 -c "import torch; print(torch.cuda.get_device_properties(0).multi_processor_count)")
# written under gpurun_out (merged back); copy them into profiles/ to commit them
python3 tools/pmc_traffic.py $OUT/fetch_$WL $OUT/write_$WL $WL "$K" $SAMPLES $OUT/pmc_$WL.json
python3 tools/pmc_deep_json.py $OUT/deep_$WL $WL "$K" $SAMPLES $CUS $OUT/pmc_deep_$WL.json
cat $OUT/kernel_stats_$WL.csv
tail -1 $OUT/kt_$WL.log
