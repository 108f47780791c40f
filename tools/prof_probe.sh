#!/bin/bash
# rocprofv3 kernel-trace + stats of the counting probe (tools/probe.py): per-kernel time split.
# usage: tools/prof_probe.sh OUTDIR [probe args...]
set -e
cd "$(dirname "$0")/.."
OUT=$1; shift
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT -o prof --output-format csv -- python3 $PWD/tools/probe.py "$@"
find $PWD/$OUT -name "*kernel_stats.csv" -exec cat {} \;
