cd $GRAFT_REPO_ROOT
O=gpurun_out/orc_shard.npy
tools/gpu_steps.sh \
 "300 fix_rr_tests.log -- python -u -m pytest tests/test_gpu_rr_repeat.py tests/test_gpu_park.py tests/test_gpu_parity.py tests/test_gpu_large.py -k 'repeat or park or russian or deep or L4 or frames_on' -x -v --timeout 300 --timeout-method thread" \
 "300 fix_oracle.log -- python -u tools/rr_shard_check.py oracle $O" \
 "120 fix_shard.log -- python -u tools/rr_shard_check.py gpu $O"
