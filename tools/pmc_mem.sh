#!/bin/bash
# Memory-hierarchy PMC passes of the quick probe: tools/pmc_mem.sh OUTDIR [probe args...]
# (honours PROBE_FLAGS / BDPT_AMD_LIB; each --pmc pass with --kernel-trace only)
set -e
cd "$(dirname "$0")/.."
OUT=$PWD/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp PROBE_QUICK=1
P="python3 $PWD/tools/probe.py $*"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_UTCL1_TRANSLATION_MISS_sum" \
           "WRITE_SIZE" "FETCH_SIZE" \
; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o p$i --output-format csv -- $P > $OUT/p$i.log 2>&1
done
python3 tools/pmc_summary.py $OUT
