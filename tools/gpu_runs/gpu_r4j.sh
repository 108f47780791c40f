cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "100 r4j_rr_probe.log -- python tools/rr_probe.py caustic 512 512 1" \
 "300 r4j_rr_tests.log -- python -u -m pytest tests/test_gpu_parity.py -x -q -k russian_roulette --timeout 200 --timeout-method thread" \
 "200 r4j_rr_l4.log -- python -u -m pytest tests/test_gpu_large.py -x -q -k L4 --timeout 190 --timeout-method thread"
