#!/bin/bash
# rocprofv3 kernel trace of one bench step under an environment setting:
# tools/kstats_env.sh TAG "VAR=v ..." [bench args]
cd "$(dirname "$0")/.."
R=$PWD; TAG=$1; E=$2; shift 2
OUT=$R/gpurun_out/kst_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for kv in $E; do export "$kv"; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- python3 $R/bench.py --no-cpu --no-parity --steps 1 --warmup 1 "$@" > $OUT/run.log 2>&1 || exit 1
find $OUT -name "*kernel_stats.csv" -exec cat {} \;
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if 'bdpt_frame_kernel' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
for r in rows[-12:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(r['Kernel_Name'][:60], s % 10**10, (e - s) / 1e6, 'ms')
PY
