cd $GRAFT_REPO_ROOT
L=$PWD/bidirectional-path-tracing_amd/lib
tools/gpu_steps.sh \
 "200 r4ae_probe.log -- env RR_PROBE_NO_COUNT=1 BDPT_AMD_LIB=$L/libbdpt_amd_cprobe.so python tools/rr_probe.py caustic 256 256 16"
