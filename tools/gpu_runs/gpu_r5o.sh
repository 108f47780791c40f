cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# slack-free interior boxes by one fma per plane (BDPT_SLAB_FMA 1: o·inv per node step
# kept out of the walk's live values; 2: left to the compiler) against the default build
: > gpurun_out/r5o.txt
run() {  # label, lib name, -- bench args
  local label=$1 lib=$2; shift 2
  local L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib/libbdpt_amd.so
  [ "$lib" != "default" ] && L=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib/libbdpt_amd_$lib.so
  BDPT_AMD_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu "$@" > gpurun_out/r5o_$label.json 2> gpurun_out/r5o_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5o_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['roofline']['kernel_ms'], d.get('parity'))" >> gpurun_out/r5o.txt
  tail -1 gpurun_out/r5o.txt
}
run c_fma1_parity slabfma1 --steps 2 --warmup 1 || exit 1
for rep in 1 2; do
  run c_def_$rep default --no-parity --steps 3 --warmup 1 || exit 1
  run c_fma1_$rep slabfma1 --no-parity --steps 3 --warmup 1 || exit 1
  run c_fma2_$rep slabfma2 --no-parity --steps 3 --warmup 1 || exit 1
done
for lib in default slabfma1 slabfma2; do
  run h_$lib $lib --no-parity --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
  run s_$lib $lib --no-parity --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
done
cat gpurun_out/r5o.txt
