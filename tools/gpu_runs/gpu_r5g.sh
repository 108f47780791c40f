cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# packed-f32 node slabs and rcp+Newton ray inverses, A/B on Caustic and synth1m
tools/gpu_steps.sh \
 "300 r5g_sweep.log -- tools/sweep_libs.sh gpurun_out/r5g_sweep.txt default pk invnr pkinv default pk invnr pkinv" \
 "300 r5g_sweep_s.log -- tools/sweep_libs.sh gpurun_out/r5g_sweep_s.txt default pk invnr pkinv -- --scene synth1m --width 1024 --height 1024 --spp 64"
