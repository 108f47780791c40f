cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "1100 r4p_gpu_tests.log -- python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread"
