cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "120 r4g_sweep.log -- tools/sweep_libs.sh gpurun_out/r4g_sweep.txt default r3 va default r3 va" && \
BDPT_DQ=1 tools/gpu_steps.sh \
 "60 r4g_probe_dq.log -- python tools/probe.py caustic 512 512 4" \
 "200 r4g_sweep_dq.log -- tools/sweep_libs.sh gpurun_out/r4g_sweep_dq.txt default dq_h2 dq_r4 dq_hi64 dq_hi384 default" \
 "120 r4g_dq_tests.log -- python -u -m pytest tests/test_gpu_dq.py -x -q --timeout 120 --timeout-method thread"
