cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# deep-scene shade threshold 36 vs 40 (synth1m), three runs each, alternating
: > gpurun_out/r5ag.txt
run() {  # label, env assignment, bench args
  local label=$1 ev=$2; shift 2
  env $ev timeout -k 10 200 python3 bench.py --no-cpu --no-parity "$@" > gpurun_out/r5ag_$label.json 2> gpurun_out/r5ag_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5ag_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])" >> gpurun_out/r5ag.txt
  tail -1 gpurun_out/r5ag.txt
}
for rep in 1 2 3; do
  run s40_$rep BDPT_SHADE_READY=40 --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
  run s36_$rep BDPT_SHADE_READY=36 --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
  run s32_$rep BDPT_SHADE_READY=32 --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1
done
run S40 BDPT_SHADE_READY=40 --scene synth1m --width 2048 --height 2048 --spp 128 --steps 1 --warmup 1 || exit 1
run S36 BDPT_SHADE_READY=36 --scene synth1m --width 2048 --height 2048 --spp 128 --steps 1 --warmup 1 || exit 1
cat gpurun_out/r5ag.txt
