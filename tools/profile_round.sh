#!/bin/bash
# Round profile of the bench workload (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats of bench.py (kernel time per launch)
#   2. --pmc FETCH_SIZE pass, 3. --pmc WRITE_SIZE pass (separate: TCC counter budget)
#   -> gpurun_out/round/{kt,fetch,write}, profiles/pmc_caustic_512x512_256spp.json
# usage: tools/profile_round.sh TAG [bench args...]
set -e
cd "$(dirname "$0")/.."
TAG=$1; shift
R=$PWD
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu $*"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $B --steps 2 --warmup 1 > $OUT/kt.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- $B --steps 1 --warmup 0 > $OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- $B --steps 1 --warmup 0 > $OUT/write.log 2>&1
cd $R
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 tools/pmc_traffic.py $OUT/fetch $OUT/write caustic_512x512_256spp "bdpt_frame_kernel<false, false>" \
  $OUT/pmc_caustic_512x512_256spp.json
cat $OUT/kernel_stats.csv
tail -1 $OUT/kt.log
