cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "300 r4s_gpu_tests.log -- python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "120 r4s_smoke.log -- python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "500 r4s_prof_caustic.log -- bash tools/profile_round.sh r4s caustic 512 512 256"
