cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "400 r4z_prof_hl.log -- bash tools/profile_round.sh r4z hardlight 512 512 1024" \
 "500 r4z_prof_synth.log -- bash tools/profile_round.sh r4z synth1m 2048 2048 512"
