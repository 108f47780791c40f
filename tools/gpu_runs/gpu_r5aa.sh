cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# the unrolled node step also after leaf iterations (BDPT_UNROLL_ANY), with traversal split 6 / 4 / 8
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
: > gpurun_out/r5aa.txt
run() {  # label, lib name, bench args
  local label=$1 lib=$2; shift 2
  local X=$L/libbdpt_amd.so
  [ "$lib" != "default" ] && X=$L/libbdpt_amd_$lib.so
  BDPT_AMD_LIB=$X timeout -k 10 200 python3 bench.py --no-cpu --no-parity "$@" > gpurun_out/r5aa_$label.json 2> gpurun_out/r5aa_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5aa_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])" >> gpurun_out/r5aa.txt
  tail -1 gpurun_out/r5aa.txt
}
for rep in 1 2; do
  for lib in default uany uany2 uany8; do run c_${lib}_$rep $lib --steps 3 --warmup 1 || exit 1; done
done
for lib in default uany uany2 uany8; do
  run h_$lib $lib --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
  run s_$lib $lib --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
done
cat gpurun_out/r5aa.txt
