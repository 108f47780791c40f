cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "600 r4n_tail.log -- bash tools/tail_sweep.sh gpurun_out/r4n_tail.txt tc0 default tc1 tc4 tc0 default -- caustic 512 512 256 1 8" \
 "400 r4n_sweep.log -- bash tools/sweep_libs.sh gpurun_out/r4n_sweep.txt tc0 default tc0 default"
