cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r4ac
tools/gpu_steps.sh \
 "400 r4ac_rr_kt.log -- rocprofv3 --kernel-trace -d gpurun_out/prof_r4ac/kt -o kt --output-format csv -- python3 tools/rr_probe.py caustic 512 512 256" \
 "400 r4ac_rr_r64.log -- env RR_PROBE_NO_COUNT=1 BDPT_PARK_ROUNDS=64 python tools/rr_probe.py caustic 512 512 256"
