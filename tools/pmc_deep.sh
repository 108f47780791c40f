#!/bin/bash
# Bottleneck counters of the frame kernel on the quick probe (tools/probe.py,
# PROBE_QUICK): one rocprofv3 --pmc pass per counter group (each within the
# per-block limits), then tools/pmc_summary.py over all passes.
# usage: tools/pmc_deep.sh OUTDIR [probe args...]
set -e
cd "$(dirname "$0")/.."
R=$PWD
OUT=$R/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp PROBE_QUICK=1
P="python3 $R/tools/probe.py $*"
cd /tmp
i=0
while read -r grp; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o p$i --output-format csv -- $P > $OUT/p$i.log 2>&1
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE
TCP_TCC_READ_REQ_LATENCY_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD
GROUPS
cd $R
python3 tools/pmc_summary.py $OUT
