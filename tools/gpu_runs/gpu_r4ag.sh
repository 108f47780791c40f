cd $GRAFT_REPO_ROOT
L=$PWD/bidirectional-path-tracing_amd/lib
tools/gpu_steps.sh \
 "300 r4ag_probe_full.log -- env RR_PROBE_NO_COUNT=1 BDPT_AMD_LIB=$L/libbdpt_amd_cp2.so python tools/rr_probe.py caustic 512 512 256"
