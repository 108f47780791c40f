cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# the extra node step only after leaf iterations (uleaf); the path tracer's split 6 / 12 and ready 48 / 60
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
: > gpurun_out/r5ae.txt
run() {  # label, lib name, bench args
  local label=$1 lib=$2; shift 2
  local X=$L/libbdpt_amd.so
  [ "$lib" != "default" ] && X=$L/libbdpt_amd_$lib.so
  BDPT_AMD_LIB=$X timeout -k 10 200 python3 bench.py --no-cpu --no-parity "$@" > gpurun_out/r5ae_$label.json 2> gpurun_out/r5ae_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5ae_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])" >> gpurun_out/r5ae.txt
  tail -1 gpurun_out/r5ae.txt
}
for rep in 1 2; do
  for lib in default uleaf; do run c_${lib}_$rep $lib --steps 3 --warmup 1 || exit 1; done
done
for lib in default uleaf; do
  run h_$lib $lib --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
  run s_$lib $lib --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
done
for rep in 1 2; do
  for lib in default ptsp6 ptsp12 ptr48 ptr60; do run p_${lib}_$rep $lib --integrator path --spp 64 --steps 5 --warmup 1 || exit 1; done
done
cat gpurun_out/r5ae.txt
