#!/bin/bash
# Per-kernel time split and PMC counters of the quick probe (tools/probe.py, PROBE_QUICK).
# usage: tools/pmc_probe.sh OUTDIR [probe args...]   (separate rocprofv3 passes, --pmc never
# combined with tracing domains other than --kernel-trace)
set -e
cd "$(dirname "$0")/.."
OUT=$PWD/$1; shift
export TMPDIR=/tmp PROBE_QUICK=1
P="python3 $PWD/tools/probe.py $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $P > $OUT.kt.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $OUT/p1 -o p1 --output-format csv -- $P > $OUT.p1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/p2 -o p2 --output-format csv -- $P > $OUT.p2.log 2>&1
find $OUT/kt -name "*kernel_stats.csv" -exec cat {} \;
