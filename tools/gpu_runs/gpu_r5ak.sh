cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# an occlusion query tests the lane's last occluder first (BDPT_OCC_CACHE); parity first
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
: > gpurun_out/r5ak.txt
BDPT_AMD_LIB=$L/libbdpt_amd_occ.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5ak_tests.log 2>&1 || { tail -5 gpurun_out/r5ak_tests.log; exit 1; }
tail -1 gpurun_out/r5ak_tests.log >> gpurun_out/r5ak.txt
run() {  # label, lib name, bench args
  local label=$1 lib=$2; shift 2
  local X=$L/libbdpt_amd.so
  [ "$lib" != "default" ] && X=$L/libbdpt_amd_$lib.so
  BDPT_AMD_LIB=$X timeout -k 10 200 python3 bench.py --no-cpu --no-parity "$@" > gpurun_out/r5ak_$label.json 2> gpurun_out/r5ak_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5ak_$label.json').read().strip().splitlines()[-1]); c=d['roofline'].get('counts_per_sample') or {}; print('$label', d['value'], d['ms_per_step'], c.get('interior_visits'), c.get('tri_tests'))" >> gpurun_out/r5ak.txt
  tail -1 gpurun_out/r5ak.txt
}
for rep in 1 2; do
  for lib in default occ; do run c_${lib}_$rep $lib --steps 3 --warmup 1 || exit 1; done
done
for lib in default occ; do
  run h_$lib $lib --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
  run s_$lib $lib --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
done
cat gpurun_out/r5ak.txt
