cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# shade threshold re-swept on the unroll-any build (BDPT_SHADE_READY env override)
: > gpurun_out/r5ac.txt
run() {  # label, env assignment or -, bench args
  local label=$1 ev=$2; shift 2
  [ "$ev" == "-" ] && ev="BDPT_NONE=1"
  env $ev timeout -k 10 200 python3 bench.py --no-cpu --no-parity "$@" > gpurun_out/r5ac_$label.json 2> gpurun_out/r5ac_$label.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5ac_$label.json').read().strip().splitlines()[-1]); print('$label', d['value'], d['ms_per_step'])" >> gpurun_out/r5ac.txt
  tail -1 gpurun_out/r5ac.txt
}
for rep in 1 2; do
  for r in def 40 48 52; do
    ev=-; [ "$r" != "def" ] && ev=BDPT_SHADE_READY=$r
    run c_${r}_$rep $ev --steps 3 --warmup 1 || exit 1
  done
done
for r in def 40 48; do ev=-; [ "$r" != "def" ] && ev=BDPT_SHADE_READY=$r; run h_$r $ev --scene hardlight --spp 1024 --steps 3 --warmup 1 || exit 1; done
for r in def 36 44; do ev=-; [ "$r" != "def" ] && ev=BDPT_SHADE_READY=$r; run s_$r $ev --scene synth1m --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 || exit 1; done
cat gpurun_out/r5ac.txt
