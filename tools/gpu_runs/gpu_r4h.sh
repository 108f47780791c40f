cd $GRAFT_REPO_ROOT
export BDPT_DQ=1
tools/gpu_steps.sh \
 "60 r4h_dq_smoke.log -- python tools/dq_smoke.py caustic 128 128 16 8" && \
tools/gpu_steps.sh \
 "120 r4h_dq_tests.log -- python -u -m pytest tests/test_gpu_dq.py -x -q --timeout 120 --timeout-method thread" \
 "60 r4h_probe_dq.log -- python tools/probe.py caustic 512 512 4" \
 "200 r4h_sweep_dq.log -- tools/sweep_libs.sh gpurun_out/r4h_sweep_dq.txt default dq_h2 dq_h3 dq_h0 default" \
 "100 r4h_rr_probe.log -- env BDPT_DQ=0 python tools/rr_probe.py caustic 512 512 1"
