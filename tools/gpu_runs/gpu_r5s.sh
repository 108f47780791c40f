cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# walk-loop trims on the sign-picked-plane default: the LDS root through the picked planes
# (lnf), the far bound from ts.best_t and one fma (far2), both (walk3); parity + KAT on walk3 first
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
: > gpurun_out/r5s.txt
BDPT_AMD_LIB=$L/libbdpt_amd_walk3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5s_tests_walk3.log 2>&1 || { tail -5 gpurun_out/r5s_tests_walk3.log; exit 1; }
tail -1 gpurun_out/r5s_tests_walk3.log >> gpurun_out/r5s.txt
run() {  # label, lib name, bench args
  local label=$1 lib=$2; shift 2
  local X=$L/libbdpt_amd.so
  [ "$lib" != "default" ] && X=$L/libbdpt_amd_$lib.so
  BDPT_AMD_LIB=$X timeout -k 10 200 python3 bench.py --no-cpu "$@" > gpurun_out/r5s_$label.json 2> gpurun_out/r5s_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5s_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['roofline']['kernel_ms'])" >> gpurun_out/r5s.txt
  tail -1 gpurun_out/r5s.txt
}
for rep in 1 2; do
  for lib in default lnf far2 walk3; do run c_${lib}_$rep $lib --no-parity --steps 3 --warmup 1 || exit 1; done
done
for lib in default lnf far2 walk3; do
  run h_$lib $lib --no-parity --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
  run s_$lib $lib --no-parity --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
done
cat gpurun_out/r5s.txt
