cd $GRAFT_REPO_ROOT
L=$PWD/bidirectional-path-tracing_amd/lib
tools/gpu_steps.sh \
 "400 r4r_sweep.log -- bash tools/sweep_libs.sh gpurun_out/r4r_sweep.txt tr0 default tr0 default -- " \
 "200 r4r_hl.log -- bash tools/sweep_libs.sh gpurun_out/r4r_hl.txt tr0 default -- --scene hardlight --spp 1024" \
 "300 r4r_deep.log -- bash tools/sweep_libs.sh gpurun_out/r4r_deep.txt default ra0 default ra0 -- --rr-depth 64 --spp 32" \
 "120 r4r_rr_default.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py caustic 256 256 16" \
 "120 r4r_rr_ra0.log -- env RR_PROBE_NO_COUNT=1 BDPT_AMD_LIB=$L/libbdpt_amd_ra0.so python tools/rr_probe.py caustic 256 256 16" \
 "120 r4r_rr_tr0.log -- env RR_PROBE_NO_COUNT=1 BDPT_AMD_LIB=$L/libbdpt_amd_tr0.so python tools/rr_probe.py caustic 256 256 16"
