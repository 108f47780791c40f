cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "300 r4l_row96.log -- python tools/rr_probe.py caustic 512 512 1 96 512"
