cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "500 r4o_sweep.log -- bash tools/sweep_libs.sh gpurun_out/r4o_sweep.txt tc0 default sc0 tc4 tc0 default sc0 tc4" \
 "400 r4o_tail.log -- bash tools/tail_sweep.sh gpurun_out/r4o_tail.txt tc0 default sc0 tc4 -- caustic 512 512 256 1 8" \
 "300 r4o_hl.log -- bash tools/sweep_libs.sh gpurun_out/r4o_hl.txt tc0 default -- --scene hardlight --spp 1024"
