cd $GRAFT_REPO_ROOT
L=$PWD/bidirectional-path-tracing_amd/lib
tools/gpu_steps.sh \
 "200 r4af_park_tests.log -- python -u -m pytest tests/test_gpu_park.py -x -q --timeout 300 --timeout-method thread" \
 "200 r4af_probe_cp2.log -- env RR_PROBE_NO_COUNT=1 BDPT_AMD_LIB=$L/libbdpt_amd_cp2.so python tools/rr_probe.py caustic 256 256 16" \
 "200 r4af_probe_lds.log -- env RR_PROBE_NO_COUNT=1 BDPT_AMD_LIB=$L/libbdpt_amd_cprobe.so python tools/rr_probe.py caustic 256 256 16" \
 "200 r4af_probe_hbm.log -- env RR_PROBE_NO_COUNT=1 BDPT_AMD_LIB=$L/libbdpt_amd_cp0.so python tools/rr_probe.py caustic 256 256 16"
