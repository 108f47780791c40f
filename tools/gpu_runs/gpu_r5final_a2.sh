cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r5
# the profiled configurations again on the committed tree (the first pass was stamped from a tree that
# carried an uncommitted source experiment; the library it ran was this one)
tools/gpu_steps.sh \
 "300 r5f_prof_caustic.log -- bash tools/profile_round.sh r5 caustic 512 512 256" \
 "300 r5f_prof_hl.log -- bash tools/profile_round.sh r5 hardlight 512 512 1024" \
 "400 r5f_prof_c1024.log -- bash tools/profile_round.sh r5 caustic 1024 1024 1024" \
 "500 r5f_prof_synth.log -- bash tools/profile_round.sh r5 synth1m 2048 2048 512"
