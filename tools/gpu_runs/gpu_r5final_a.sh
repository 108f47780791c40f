cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r5
# the final round-5 build: GPU suite, smoke, the profiled configurations (configs[1..4] on one GPU),
# stamped PMC summaries copied into profiles/ on the box so the bench lines of gpu_r5final_b.sh carry them
tools/gpu_steps.sh \
 "400 r5f_gpu_tests.log -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "120 r5f_smoke.log -- python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "300 r5f_prof_caustic.log -- bash tools/profile_round.sh r5 caustic 512 512 256" \
 "300 r5f_prof_hl.log -- bash tools/profile_round.sh r5 hardlight 512 512 1024" \
 "400 r5f_prof_c1024.log -- bash tools/profile_round.sh r5 caustic 1024 1024 1024" \
 "500 r5f_prof_synth.log -- bash tools/profile_round.sh r5 synth1m 2048 2048 512"
