cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# runtime shade threshold / traversal split (variant library rtsplit): synth1m and Caustic
export BDPT_AMD_LIB=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib/libbdpt_amd_rtsplit.so
: > gpurun_out/r5n.txt
run() {  # label, env..., -- bench args
  local label=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu --no-parity --steps 3 --warmup 1 $BARGS > gpurun_out/r5n_$label.json 2> gpurun_out/r5n_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5n_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['roofline']['kernel_ms'])" >> gpurun_out/r5n.txt
}
BARGS="--scene synth1m --width 1024 --height 1024 --spp 64"
for rep in 1 2; do
  run s_r40_t6 BDPT_SHADE_READY=40 BDPT_TRAV_SPLIT_RT=6 || exit 1
  run s_r40_t4 BDPT_SHADE_READY=40 BDPT_TRAV_SPLIT_RT=4 || exit 1
  run s_r40_t5 BDPT_SHADE_READY=40 BDPT_TRAV_SPLIT_RT=5 || exit 1
  run s_r36_t4 BDPT_SHADE_READY=36 BDPT_TRAV_SPLIT_RT=4 || exit 1
  run s_r40_t3 BDPT_SHADE_READY=40 BDPT_TRAV_SPLIT_RT=3 || exit 1
done
BARGS=""
for rep in 1 2; do
  run c_r44_t6 BDPT_SHADE_READY=44 BDPT_TRAV_SPLIT_RT=6 || exit 1
  run c_r44_t5 BDPT_SHADE_READY=44 BDPT_TRAV_SPLIT_RT=5 || exit 1
  run c_r44_t7 BDPT_SHADE_READY=44 BDPT_TRAV_SPLIT_RT=7 || exit 1
done
cat gpurun_out/r5n.txt
