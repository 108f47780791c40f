cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r4ad
tools/gpu_steps.sh \
 "200 r4ad_park_tests.log -- python -u -m pytest tests/test_gpu_park.py tests/test_gpu_parity.py -k 'park or russian' -x -q --timeout 300 --timeout-method thread" \
 "400 r4ad_rr_kt.log -- RR_PROBE_NO_COUNT=1 rocprofv3 --kernel-trace -d gpurun_out/prof_r4ad/kt -o kt --output-format csv -- python3 tools/rr_probe.py caustic 512 512 256"
