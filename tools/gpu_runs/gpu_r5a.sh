cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# round 5, first call: the suite after the dq removal, the ring tag and the RR wave walks in turn;
# the connection-task histogram (counting passes); the default bench; one RR Caustic frame
tools/gpu_steps.sh \
 "400 r5a_gpu_tests.log -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "120 r5a_smoke.log -- python -c 'import __graft_entry__ as g; g.smoke()'" \
 "120 r5a_probe_caustic.log -- python tools/probe.py caustic 512 512 16" \
 "120 r5a_probe_hardlight.log -- python tools/probe.py hardlight 512 512 64" \
 "120 r5a_probe_synth1m.log -- python tools/probe.py synth1m 1024 1024 16" \
 "200 r5a_bench.json -- python3 bench.py --steps 20 --warmup 2" \
 "150 r5a_rr_hl.log -- python tools/rr_probe.py hardlight 512 512 64" \
 "200 r5a_rr_caustic.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py caustic 512 512 256"
