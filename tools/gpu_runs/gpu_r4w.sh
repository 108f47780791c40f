cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "300 r4w_tail.log -- bash tools/tail_sweep.sh gpurun_out/r4w_tail.txt default tf4 tf5 tf7 default tf4 tf5 tf7 -- caustic 512 512 256 1 8" \
 "300 r4w_sweep.log -- bash tools/sweep_libs.sh gpurun_out/r4w_sweep.txt default tf4 tf5 tf7"
