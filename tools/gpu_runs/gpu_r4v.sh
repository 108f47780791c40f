cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "300 r4v_tail.log -- bash tools/tail_sweep.sh gpurun_out/r4v_tail.txt default ts2 ts1 default ts2 ts1 -- caustic 512 512 256 1 8" \
 "300 r4v_sweep.log -- bash tools/sweep_libs.sh gpurun_out/r4v_sweep.txt default ts2 ts1 default ts2 ts1"
