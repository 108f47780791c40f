cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# a leaf step after node iterations too (BDPT_LEAF_ANY), traversal split 8 / 10 / 6, against the default
L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib
: > gpurun_out/r5ad.txt
run() {  # label, lib name, bench args
  local label=$1 lib=$2; shift 2
  local X=$L/libbdpt_amd.so
  [ "$lib" != "default" ] && X=$L/libbdpt_amd_$lib.so
  BDPT_AMD_LIB=$X timeout -k 10 200 python3 bench.py --no-cpu --no-parity "$@" > gpurun_out/r5ad_$label.json 2> gpurun_out/r5ad_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5ad_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])" >> gpurun_out/r5ad.txt
  tail -1 gpurun_out/r5ad.txt
}
for rep in 1 2; do
  for lib in default lany lany10 lany6; do run c_${lib}_$rep $lib --steps 3 --warmup 1 || exit 1; done
done
for lib in default lany lany10 lany6; do
  run h_$lib $lib --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
  run s_$lib $lib --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
done
cat gpurun_out/r5ad.txt
