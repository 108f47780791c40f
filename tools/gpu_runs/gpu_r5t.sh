cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# on the walk3 default: the shade threshold read before the walk loop (rh); schedule constants
# re-swept (walk unroll 2, traversal split 5 / 8, shade-ready 40 / 48 through the env override)
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
: > gpurun_out/r5t.txt
run() {  # label, lib name, env assignment or -, bench args
  local label=$1 lib=$2 ev=$3; shift 3
  local X=$L/libbdpt_amd.so
  [ "$lib" != "default" ] && X=$L/libbdpt_amd_$lib.so
  [ "$ev" == "-" ] && ev="BDPT_NONE=1"
  env BDPT_AMD_LIB=$X $ev timeout -k 10 200 python3 bench.py --no-cpu "$@" > gpurun_out/r5t_$label.json 2> gpurun_out/r5t_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5t_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['roofline']['kernel_ms'])" >> gpurun_out/r5t.txt
  tail -1 gpurun_out/r5t.txt
}
for rep in 1 2; do
  run c_def_$rep default - --no-parity --steps 3 --warmup 1 || exit 1
  run c_rh_$rep rh - --no-parity --steps 3 --warmup 1 || exit 1
  run c_unr2_$rep unr2 - --no-parity --steps 3 --warmup 1 || exit 1
  run c_sp5_$rep sp5 - --no-parity --steps 3 --warmup 1 || exit 1
  run c_sp8_$rep sp8 - --no-parity --steps 3 --warmup 1 || exit 1
  run c_r40_$rep default BDPT_SHADE_READY=40 --no-parity --steps 3 --warmup 1 || exit 1
  run c_r48_$rep default BDPT_SHADE_READY=48 --no-parity --steps 3 --warmup 1 || exit 1
done
for lib in default rh unr2 sp5 sp8; do
  run h_$lib $lib - --no-parity --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
  run s_$lib $lib - --no-parity --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
done
run s_r36 default BDPT_SHADE_READY=36 --no-parity --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
run s_r44 default BDPT_SHADE_READY=44 --no-parity --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
run h_r40 default BDPT_SHADE_READY=40 --no-parity --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
run h_r48 default BDPT_SHADE_READY=48 --no-parity --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
cat gpurun_out/r5t.txt
