set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 1 --warmup 0 --spp 16"
cd /tmp
timeout -k 10 300 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d $GRAFT_REPO_ROOT/gpurun_out/pmc1 -o p1 --output-format csv -- $B > $GRAFT_REPO_ROOT/gpurun_out/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/pmc2 -o p2 --output-format csv -- $B > $GRAFT_REPO_ROOT/gpurun_out/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/pmc3 -o p3 --output-format csv -- $B > $GRAFT_REPO_ROOT/gpurun_out/pmc3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_FLAT SQ_WAIT_INST_ANY -d $GRAFT_REPO_ROOT/gpurun_out/pmc4 -o p4 --output-format csv -- $B > $GRAFT_REPO_ROOT/gpurun_out/pmc4.log 2>&1
