cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "900 r4k_rr_full.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py caustic 512 512 256"
