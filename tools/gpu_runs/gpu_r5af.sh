cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# Russian roulette: express waves with 2-4 long walks walk them at once in groups of 32 / 16 lanes
# (BDPT_COOP_GROUPS): RR tests on it, then RR Caustic frames, default and grouped, alternating
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
: > gpurun_out/r5af.txt
BDPT_AMD_LIB=$L/libbdpt_amd_cgrp.so timeout -k 10 400 python -u -m pytest tests -m gpu -k "rr or roulette or RR" -x -q --timeout 300 --timeout-method thread > gpurun_out/r5af_rr_tests.log 2>&1 || { tail -5 gpurun_out/r5af_rr_tests.log; exit 1; }
tail -1 gpurun_out/r5af_rr_tests.log >> gpurun_out/r5af.txt
run() {  # label, lib name, bench args
  local label=$1 lib=$2; shift 2
  local X=$L/libbdpt_amd.so
  [ "$lib" != "default" ] && X=$L/libbdpt_amd_$lib.so
  BDPT_AMD_LIB=$X timeout -k 10 300 python3 bench.py --no-cpu "$@" > gpurun_out/r5af_$label.json 2> gpurun_out/r5af_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5af_$label.json').read().strip().splitlines()[-1]); r=d['russian_roulette']; print('$label', d['value'], d['ms_per_step'], r['express_iters_1_2to4_more_per_step'], (d.get('parity') or {}).get('max_rel_l2'))" >> gpurun_out/r5af.txt
  tail -1 gpurun_out/r5af.txt
}
run rrc_cgrp_par cgrp --russian-roulette --steps 1 --warmup 0 || exit 1
for rep in 1 2; do
  run rrc_def_$rep default --no-parity --russian-roulette --steps 1 --warmup 0 || exit 1
  run rrc_cgrp_$rep cgrp --no-parity --russian-roulette --steps 1 --warmup 0 || exit 1
done
run rrh_cgrp cgrp --no-parity --russian-roulette --scene hardlight --spp 1024 --steps 2 --warmup 1 || exit 1
cat gpurun_out/r5af.txt
