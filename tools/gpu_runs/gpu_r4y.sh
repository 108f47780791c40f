cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "300 r4y_gpu_tests.log -- python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "120 r4y_smoke.log -- python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "400 r4y_prof_caustic.log -- bash tools/profile_round.sh r4y caustic 512 512 256"
