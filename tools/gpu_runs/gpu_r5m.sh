cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# new defaults (shade-ready 44, traversal split 6) against 40 / 36 and split 4 / 5
tools/gpu_steps.sh \
 "400 r5m_sweep.log -- tools/sweep_libs.sh gpurun_out/r5m_sweep.txt default sr40 sr36 ts4 ts5 default sr40 sr36 ts4 ts5" \
 "300 r5m_sweep_s.log -- tools/sweep_libs.sh gpurun_out/r5m_sweep_s.txt default sr40 sr36 ts4 ts5 -- --scene synth1m --width 1024 --height 1024 --spp 64" \
 "200 r5m_sweep_hl.log -- tools/sweep_libs.sh gpurun_out/r5m_sweep_hl.txt default sr40 ts4 ts5 -- --scene hardlight --spp 1024"
