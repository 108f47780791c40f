cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# near / far planes picked by the ray's direction signs at the node load (BDPT_SLAB_SIGN 1: the
# sign offsets formed per node step; 2: left to the compiler) against the fma-slab default;
# (2m: with the merged near / far hit test, BDPT_HIT_MERGE); the parity and KAT suites on sign2m first
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
: > gpurun_out/r5r.txt
BDPT_AMD_LIB=$L/libbdpt_amd_sign2m.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5r_tests_sign2m.log 2>&1 || { tail -5 gpurun_out/r5r_tests_sign2m.log; exit 1; }
tail -1 gpurun_out/r5r_tests_sign2m.log >> gpurun_out/r5r.txt
run() {  # label, lib name, bench args
  local label=$1 lib=$2; shift 2
  local X=$L/libbdpt_amd.so
  [ "$lib" != "default" ] && X=$L/libbdpt_amd_$lib.so
  BDPT_AMD_LIB=$X timeout -k 10 200 python3 bench.py --no-cpu "$@" > gpurun_out/r5r_$label.json 2> gpurun_out/r5r_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5r_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['roofline']['kernel_ms'])" >> gpurun_out/r5r.txt
  tail -1 gpurun_out/r5r.txt
}
for rep in 1 2; do
  run c_def_$rep default --no-parity --steps 3 --warmup 1 || exit 1
  run c_sign1_$rep sign1 --no-parity --steps 3 --warmup 1 || exit 1
  run c_sign2_$rep sign2 --no-parity --steps 3 --warmup 1 || exit 1
  run c_sign2m_$rep sign2m --no-parity --steps 3 --warmup 1 || exit 1
done
for lib in default sign1 sign2 sign2m; do
  run h_$lib $lib --no-parity --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
  run s_$lib $lib --no-parity --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
done
cat gpurun_out/r5r.txt
