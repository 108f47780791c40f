#!/bin/bash
# One rocprofv3 --pmc pass over a short bench run, summarised per launch of the
# timed frame kernel: tools/pmc_pass.sh TAG "COUNTER ..." [bench args]
# -> gpurun_out/pmc_TAG/summary.json (counter totals per launch and per sample)
cd "$(dirname "$0")/.."
TAG=$1 CTRS=$2; shift 2
R=$PWD OUT=$PWD/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/raw -o p --output-format csv -- \
  python3 $R/bench.py --no-cpu --no-parity --steps 1 --warmup 0 "$@" > $OUT/run.log 2>&1 || exit $?
cd $R
python3 tools/pmc_counters.py $OUT/raw "bdpt_frame_kernel<false, false, false>" $OUT/run.log > $OUT/summary.json
cat $OUT/summary.json
