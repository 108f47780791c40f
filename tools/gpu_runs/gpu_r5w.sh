cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# traversal-tree build parameters re-swept on the sign-picked-plane build (host env, no rebuild):
# triangle leaf size 3 / 2 (4), SAH node cost 0.5 / 0.7 (1.0), collapse DP node cost 0.5 / 0.7 / 1.5 (1.0)
: > gpurun_out/r5w.txt
run() {  # label, env assignment or -, bench args
  local label=$1 ev=$2; shift 2
  [ "$ev" == "-" ] && ev="BDPT_NONE=1"
  env $ev timeout -k 10 250 python3 bench.py --no-cpu --no-parity "$@" > gpurun_out/r5w_$label.json 2> gpurun_out/r5w_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5w_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['roofline']['kernel_ms'])" >> gpurun_out/r5w.txt
  tail -1 gpurun_out/r5w.txt
}
for rep in 1 2; do
  run c_def_$rep - --steps 3 --warmup 1 || exit 1
  run c_leaf3_$rep BDPT_TRI_LEAF_MAX=3 --steps 3 --warmup 1 || exit 1
  run c_leaf2_$rep BDPT_TRI_LEAF_MAX=2 --steps 3 --warmup 1 || exit 1
  run c_snc05_$rep BDPT_SAH_NODE_COST=0.5 --steps 3 --warmup 1 || exit 1
  run c_snc07_$rep BDPT_SAH_NODE_COST=0.7 --steps 3 --warmup 1 || exit 1
  run c_dnc05_$rep BDPT_DP_NODE_COST=0.5 --steps 3 --warmup 1 || exit 1
  run c_dnc07_$rep BDPT_DP_NODE_COST=0.7 --steps 3 --warmup 1 || exit 1
  run c_dnc15_$rep BDPT_DP_NODE_COST=1.5 --steps 3 --warmup 1 || exit 1
done
for cfg in "def -" "leaf3 BDPT_TRI_LEAF_MAX=3" "snc07 BDPT_SAH_NODE_COST=0.7" "dnc07 BDPT_DP_NODE_COST=0.7"; do
  set -- $cfg
  run h_$1 $2 --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1
  run s_$1 $2 --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
done
cat gpurun_out/r5w.txt
