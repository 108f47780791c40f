cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# schedule constants re-swept on the fast-weights build
tools/gpu_steps.sh \
 "400 r5k_sweep.log -- tools/sweep_libs.sh gpurun_out/r5k_sweep.txt default sr44 sr52 ts6 wu0 default sr44 sr52 ts6 wu0"
