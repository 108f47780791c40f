cd $GRAFT_REPO_ROOT
L=$PWD/bidirectional-path-tracing_amd/lib
tools/gpu_steps.sh \
 "200 fix3_rr_repeat.log -- python -u -m pytest tests/test_gpu_rr_repeat.py -q --timeout 300 --timeout-method thread" \
 "200 fix3_bug_control.log -- env BDPT_AMD_LIB=$L/libbdpt_amd_bug.so python -u -m pytest tests/test_gpu_rr_repeat.py -q --timeout 300 --timeout-method thread"
