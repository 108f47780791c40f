cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# the path tracer and direct integrator on the slack-free interior test (host node_slack_needed
# per render, pt_frame_kernel<.., SLACK>) against the slack test everywhere (ptslack); their GPU tests
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
: > gpurun_out/r5u.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -k "path or direct or pt_ or Path or Direct" -x -q --timeout 120 --timeout-method thread > gpurun_out/r5u_tests.log 2>&1 || { tail -5 gpurun_out/r5u_tests.log; exit 1; }
tail -1 gpurun_out/r5u_tests.log >> gpurun_out/r5u.txt
run() {  # label, lib name, bench args
  local label=$1 lib=$2; shift 2
  local X=$L/libbdpt_amd.so
  [ "$lib" != "default" ] && X=$L/libbdpt_amd_$lib.so
  BDPT_AMD_LIB=$X timeout -k 10 200 python3 bench.py --no-cpu "$@" > gpurun_out/r5u_$label.json 2> gpurun_out/r5u_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5u_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])" >> gpurun_out/r5u.txt
  tail -1 gpurun_out/r5u.txt
}
for rep in 1 2; do
  run p_def_$rep default --no-parity --integrator path --spp 64 --steps 5 --warmup 1 || exit 1
  run p_slack_$rep ptslack --no-parity --integrator path --spp 64 --steps 5 --warmup 1 || exit 1
  run d_def_$rep default --no-parity --integrator direct --spp 64 --steps 5 --warmup 1 || exit 1
  run d_slack_$rep ptslack --no-parity --integrator direct --spp 64 --steps 5 --warmup 1 || exit 1
done
run p_def_parity default --integrator path --spp 64 --steps 2 --warmup 1 || exit 1
cat gpurun_out/r5u.txt
