cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# new defaults (shade-ready 44, traversal split 6, fast Phong pow) against 40 / 36, split 4 / 5, exact pow;
# WRITE_SIZE of the default build against probes without camera-splat atomics / light-vertex stores
tools/gpu_steps.sh \
 "100 r5m_kat.log -- python -u -m pytest tests/test_gpu_kat.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 'golden or kat or hardlight'" \
 "400 r5m_sweep.log -- tools/sweep_libs.sh gpurun_out/r5m_sweep.txt default sr40 sr36 ts4 ts5 default sr40 sr36 ts4 ts5" \
 "300 r5m_sweep_s.log -- tools/sweep_libs.sh gpurun_out/r5m_sweep_s.txt default sr40 ts4 ts5 -- --scene synth1m --width 1024 --height 1024 --spp 64" \
 "200 r5m_sweep_hl.log -- tools/sweep_libs.sh gpurun_out/r5m_sweep_hl.txt default exactpow sr40 ts4 default exactpow -- --scene hardlight --spp 1024" \
 "100 r5m_w_default.log -- bash tools/pmc_write_lib.sh default" \
 "100 r5m_w_nosplat.log -- bash tools/pmc_write_lib.sh nosplat" \
 "100 r5m_w_nolvst.log -- bash tools/pmc_write_lib.sh nolvst"
