cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# coop_closest on the sign-picked planes (BDPT_COOP_NF, the RR build's cooperative walks): RR tests,
# then RR Caustic / HardLight A/B; the translated-scene path / direct parity cases on the default
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
: > gpurun_out/r5z.txt
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "translated" -x -q --timeout 120 --timeout-method thread > gpurun_out/r5z_translated.log 2>&1 || { tail -5 gpurun_out/r5z_translated.log; exit 1; }
tail -1 gpurun_out/r5z_translated.log >> gpurun_out/r5z.txt
BDPT_AMD_LIB=$L/libbdpt_amd_coopnf.so timeout -k 10 400 python -u -m pytest tests -m gpu -k "rr or roulette or RR" -x -q --timeout 300 --timeout-method thread > gpurun_out/r5z_rr_tests.log 2>&1 || { tail -5 gpurun_out/r5z_rr_tests.log; exit 1; }
tail -1 gpurun_out/r5z_rr_tests.log >> gpurun_out/r5z.txt
run() {  # label, lib name, bench args
  local label=$1 lib=$2; shift 2
  local X=$L/libbdpt_amd.so
  [ "$lib" != "default" ] && X=$L/libbdpt_amd_$lib.so
  BDPT_AMD_LIB=$X timeout -k 10 300 python3 bench.py --no-cpu --no-parity "$@" > gpurun_out/r5z_$label.json 2> gpurun_out/r5z_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5z_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])" >> gpurun_out/r5z.txt
  tail -1 gpurun_out/r5z.txt
}
for lib in default coopnf default coopnf; do
  run rrc_$lib $lib --russian-roulette --steps 1 --warmup 0 || exit 1
done
for lib in default coopnf; do
  run rrh_$lib $lib --russian-roulette --scene hardlight --spp 1024 --steps 2 --warmup 1 || exit 1
done
cat gpurun_out/r5z.txt
