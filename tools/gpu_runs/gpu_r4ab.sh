cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "400 r4ab_park_tests.log -- python -u -m pytest tests/test_gpu_park.py -x -v --timeout 300 --timeout-method thread" \
 "300 r4ab_gpu_tests.log -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "200 r4ab_rr_256.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py caustic 256 256 16" \
 "400 r4ab_rr_full.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py caustic 512 512 256"
