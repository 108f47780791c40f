cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# the root's grandchildren in LDS too (BDPT_ROOT_L3, with a 6-entry LDS stack to fit) against the
# default and the 6-entry stack alone; parity + KAT + large suites on l3 first
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
: > gpurun_out/r5ah.txt
BDPT_AMD_LIB=$L/libbdpt_amd_l3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_large.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5ah_tests.log 2>&1 || { tail -5 gpurun_out/r5ah_tests.log; exit 1; }
tail -1 gpurun_out/r5ah_tests.log >> gpurun_out/r5ah.txt
run() {  # label, lib name, bench args
  local label=$1 lib=$2; shift 2
  local X=$L/libbdpt_amd.so
  [ "$lib" != "default" ] && X=$L/libbdpt_amd_$lib.so
  BDPT_AMD_LIB=$X timeout -k 10 200 python3 bench.py --no-cpu --no-parity "$@" > gpurun_out/r5ah_$label.json 2> gpurun_out/r5ah_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5ah_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])" >> gpurun_out/r5ah.txt
  tail -1 gpurun_out/r5ah.txt
}
for rep in 1 2; do
  for lib in default l3 s6; do run c_${lib}_$rep $lib --steps 3 --warmup 1 || exit 1; done
done
for lib in default l3 s6; do
  run h_$lib $lib --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
  run s_$lib $lib --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
done
run p_default default --integrator path --spp 64 --steps 5 --warmup 1 || exit 1
run p_l3 l3 --integrator path --spp 64 --steps 5 --warmup 1 || exit 1
cat gpurun_out/r5ah.txt
