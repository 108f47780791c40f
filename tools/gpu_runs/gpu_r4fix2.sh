cd $GRAFT_REPO_ROOT
L=$PWD/bidirectional-path-tracing_amd/lib
tools/gpu_steps.sh \
 "300 fix2_rr_tests.log -- python -u -m pytest tests/test_gpu_rr_repeat.py tests/test_gpu_park.py tests/test_gpu_parity.py tests/test_gpu_large.py -k 'repeat or park or russian or deep or L4 or frames_on' -x -q --timeout 300 --timeout-method thread" \
 "200 fix2_bug_control.log -- env BDPT_AMD_LIB=$L/libbdpt_amd_bug.so python -u -m pytest tests/test_gpu_rr_repeat.py -q --timeout 300 --timeout-method thread"
