cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_fc
# the final build after the ring-cursor fix: GPU suite, smoke, the three profiled configurations,
# every bench line (profiles copied into profiles/ on the box first so bench.py stamps them)
tools/gpu_steps.sh \
 "300 fc_gpu_tests.log -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "120 fc_smoke.log -- python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "300 fc_prof_caustic.log -- bash tools/profile_round.sh fc caustic 512 512 256" \
 "300 fc_prof_hl.log -- bash tools/profile_round.sh fc hardlight 512 512 1024" \
 "400 fc_prof_synth.log -- bash tools/profile_round.sh fc synth1m 2048 2048 512" \
 "20 fc_copy.log -- cp gpurun_out/prof_fc/pmc_*.json profiles/" \
 "200 fc_bench.json -- python3 bench.py --steps 20 --warmup 2" \
 "200 fc_bench_hardlight_512x512_1024spp.json -- python3 bench.py --scene hardlight --spp 1024 --steps 5 --warmup 1" \
 "200 fc_bench_caustic_1024x1024_1024spp.json -- python3 bench.py --width 1024 --height 1024 --spp 1024 --steps 1 --warmup 1" \
 "250 fc_bench_synth1m_2048x2048_512spp.json -- python3 bench.py --scene synth1m --width 2048 --height 2048 --spp 512 --steps 1 --warmup 1" \
 "150 fc_bench_path_caustic_512x512_64spp.json -- python3 bench.py --integrator path --spp 64 --steps 5 --warmup 1" \
 "150 fc_bench_direct_caustic_512x512_64spp.json -- python3 bench.py --integrator direct --spp 64 --steps 5 --warmup 1" \
 "200 fc_bench_rr_hardlight_512x512_1024spp.json -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fc/kt_rr_hl -o kt --output-format csv -- python3 bench.py --russian-roulette --scene hardlight --spp 1024 --steps 2 --warmup 1" \
 "300 fc_bench_rr.json -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fc/kt_rr -o kt --output-format csv -- python3 bench.py --russian-roulette --steps 1 --warmup 0"
