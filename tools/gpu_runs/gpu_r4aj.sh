cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "300 r4aj_rr_tests.log -- python -u -m pytest tests/test_gpu_park.py tests/test_gpu_parity.py tests/test_gpu_large.py -k 'park or russian or L4' -x -q --timeout 300 --timeout-method thread" \
 "300 r4aj_full_nopark.log -- env RR_PROBE_NO_COUNT=1 BDPT_PARK_DEPTH=0 python tools/rr_probe.py caustic 512 512 256" \
 "300 r4aj_full_park.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py caustic 512 512 256"
