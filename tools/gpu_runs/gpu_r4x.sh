cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "300 r4x_sweep.log -- bash tools/sweep_libs.sh gpurun_out/r4x_sweep.txt c64 default c64 default" \
 "200 r4x_hl.log -- bash tools/sweep_libs.sh gpurun_out/r4x_hl.txt c64 default -- --scene hardlight --spp 1024"
