cd $GRAFT_REPO_ROOT
# the round-end commands as the driver runs them (default bench line, smoke), then two more RR frames
tools/gpu_steps.sh \
 "300 last_bench_default.json -- python3 bench.py" \
 "120 last_smoke.log -- python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "200 last_rr1.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py caustic 512 512 256" \
 "200 last_rr2.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py caustic 512 512 256"
