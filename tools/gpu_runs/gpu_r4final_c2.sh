cd $GRAFT_REPO_ROOT
L=$PWD/bidirectional-path-tracing_amd/lib
tools/gpu_steps.sh \
 "200 fc_rr_repeat.log -- python -u -m pytest tests/test_gpu_rr_repeat.py -q --timeout 300 --timeout-method thread" \
 "200 fc_bug_control.log -- env BDPT_AMD_LIB=$L/libbdpt_amd_bug.so python -u -m pytest tests/test_gpu_rr_repeat.py -q --timeout 300 --timeout-method thread" \
 "20 fc_rm_bug.log -- rm -f $L/libbdpt_amd_bug.so"
bash tools/gpu_runs/gpu_r4final_c.sh
