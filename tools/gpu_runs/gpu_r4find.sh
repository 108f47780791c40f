cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "600 find_rr_hl.log -- python -u tools/rr_find.py hardlight 512 512 1024 2 20 1"
