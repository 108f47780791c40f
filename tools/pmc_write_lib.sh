#!/bin/bash
# WRITE_SIZE of the frame kernel for a variant library: tools/pmc_write_lib.sh NAME
cd "$(dirname "$0")/.."
R=$PWD; N=$1
OUT=$R/gpurun_out/pmcw_$N
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$N" == "default" ]; then export BDPT_AMD_LIB=$R/bidirectional-path-tracing_amd/lib/libbdpt_amd.so
else export BDPT_AMD_LIB=$R/bidirectional-path-tracing_amd/lib/libbdpt_amd_$N.so; fi
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT -o w --output-format csv -- python3 $R/bench.py --no-cpu --no-parity --steps 1 --warmup 0 > $OUT/run.log 2>&1 || exit 1
f=$(find $OUT -name "*counter_collection.csv" | head -1)
python3 - "$f" "$N" <<'PY'
import csv, sys
tot = {}
for r in csv.DictReader(open(sys.argv[1])):
    if 'bdpt_frame_kernel<false, false, false>' in r['Kernel_Name']:
        tot[r['Dispatch_Id']] = tot.get(r['Dispatch_Id'], 0) + float(r['Counter_Value'])
print(sys.argv[2], 'WRITE_SIZE GB per launch:', [round(v * 1024 / 1e9, 2) for v in tot.values()])
PY
