cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# more Russian-roulette Caustic frames on the final build (grouped long walks): the frame-time spread
: > gpurun_out/r5ai.txt
for rep in 1 2 3 4; do
  timeout -k 10 300 python3 bench.py --russian-roulette --steps 1 --warmup 0 --no-cpu --no-parity > gpurun_out/r5ai_rr_$rep.json 2> gpurun_out/r5ai_rr_$rep.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r5ai_rr_$rep.json').read().strip().splitlines()[-1]); r=d['russian_roulette']; print('rr_$rep', d['ms_per_step'], r['express_iters_1_2to4_more_per_step'], r['long_walks_per_wave_max_per_step'])" >> gpurun_out/r5ai.txt
  tail -1 gpurun_out/r5ai.txt
done
cat gpurun_out/r5ai.txt
