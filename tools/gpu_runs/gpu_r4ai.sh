cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$PWD/bidirectional-path-tracing_amd/lib
mkdir -p gpurun_out/prof_r4ai
tools/gpu_steps.sh \
 "300 r4ai_probe_full.log -- BDPT_AMD_LIB=$L/libbdpt_amd_cprobe.so RR_PROBE_NO_COUNT=1 rocprofv3 --kernel-trace -d gpurun_out/prof_r4ai/kt -o kt --output-format csv -- python3 tools/rr_probe.py caustic 512 512 256"
