cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# shade-ready threshold 40 / 42 / 44 (+ traversal split 6), Caustic and HardLight
tools/gpu_steps.sh \
 "400 r5l_sweep.log -- tools/sweep_libs.sh gpurun_out/r5l_sweep.txt default sr40 sr42 sr44 sr44ts6 default sr40 sr42 sr44 sr44ts6" \
 "200 r5l_sweep_hl.log -- tools/sweep_libs.sh gpurun_out/r5l_sweep_hl.txt default sr44 sr44ts6 -- --scene hardlight --spp 1024" \
 "200 r5l_sweep_s.log -- tools/sweep_libs.sh gpurun_out/r5l_sweep_s.txt default sr44 sr44ts6 -- --scene synth1m --width 1024 --height 1024 --spp 64"
