cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "60 r4d_dq_smoke.log -- python tools/dq_smoke.py" \
 "60 r4d_dq_smoke2.log -- python tools/dq_smoke.py caustic 128 128 16 8" && \
tools/gpu_steps.sh \
 "300 r4d_dq_tests.log -- python -u -m pytest tests/test_gpu_dq.py -x -v --timeout 120 --timeout-method thread" \
 "120 r4d_dq_bench.log -- BDPT_DQ=1 python bench.py --no-cpu --no-parity --steps 3 --warmup 1"
