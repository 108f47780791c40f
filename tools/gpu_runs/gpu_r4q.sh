cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "400 r4q_gpu_tests.log -- python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 r4q_rr_default.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py caustic 512 512 16" \
 "200 r4q_rr_ra0.log -- env RR_PROBE_NO_COUNT=1 BDPT_AMD_LIB=$PWD/bidirectional-path-tracing_amd/lib/libbdpt_amd_ra0.so python tools/rr_probe.py caustic 512 512 16" \
 "300 r4q_deep.log -- bash tools/sweep_libs.sh gpurun_out/r4q_deep.txt default ra0 default ra0 -- --rr-depth 64 --spp 32"
