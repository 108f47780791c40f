cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# the full GPU suite and smoke on the final tree (after the host's deep-scene threshold change)
tools/gpu_steps.sh \
 "400 r5l_gpu_tests.log -- python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "120 r5l_smoke.log -- python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "200 r5l_bench.json -- python3 bench.py"
