cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# the walk's stack pointer as the byte offset of its top entry row (BDPT_SP_SCALED; one shift-add per
# push / pop, default kernel spills 4 -> 2): parity + KAT + path / direct suites on it, then the A/B
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
: > gpurun_out/r5y.txt
BDPT_AMD_LIB=$L/libbdpt_amd_sps.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_large.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5y_tests.log 2>&1 || { tail -5 gpurun_out/r5y_tests.log; exit 1; }
tail -1 gpurun_out/r5y_tests.log >> gpurun_out/r5y.txt
run() {  # label, lib name, bench args
  local label=$1 lib=$2; shift 2
  local X=$L/libbdpt_amd.so
  [ "$lib" != "default" ] && X=$L/libbdpt_amd_$lib.so
  BDPT_AMD_LIB=$X timeout -k 10 200 python3 bench.py --no-cpu --no-parity "$@" > gpurun_out/r5y_$label.json 2> gpurun_out/r5y_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5y_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])" >> gpurun_out/r5y.txt
  tail -1 gpurun_out/r5y.txt
}
for rep in 1 2 3; do
  run c_def_$rep default --steps 3 --warmup 1 || exit 1
  run c_sps_$rep sps --steps 3 --warmup 1 || exit 1
done
for lib in default sps; do
  run h_$lib $lib --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
  run s_$lib $lib --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
  run p_$lib $lib --integrator path --spp 64 --steps 5 --warmup 1 || exit 1
done
cat gpurun_out/r5y.txt
