cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# the fifth final round-5 build (+ node steps after leaf iterations, split 8, path unroll, RR grouped walks): GPU suite,
# smoke, the profiled configurations (stamps copied into profiles/ on the box so the bench lines
# after them carry them), then every bench line
P=gpurun_out/prof_r5e
tools/gpu_steps.sh \
 "400 r5j_gpu_tests.log -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "120 r5j_smoke.log -- python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "300 r5j_prof_caustic.log -- bash tools/profile_round.sh r5e caustic 512 512 256" \
 "300 r5j_prof_hl.log -- bash tools/profile_round.sh r5e hardlight 512 512 1024" \
 "400 r5j_prof_c1024.log -- bash tools/profile_round.sh r5e caustic 1024 1024 1024" \
 "500 r5j_prof_synth.log -- bash tools/profile_round.sh r5e synth1m 2048 2048 512" \
 "30 r5j_copy.log -- cp $P/pmc_*.json profiles/ && ls -la profiles/pmc_*" \
 "200 r5j_bench.json -- python3 bench.py --steps 20 --warmup 2" \
 "200 r5j_bench_hardlight_512x512_1024spp.json -- python3 bench.py --scene hardlight --spp 1024 --steps 5 --warmup 1" \
 "250 r5j_bench_caustic_1024x1024_1024spp.json -- python3 bench.py --width 1024 --height 1024 --spp 1024 --steps 1 --warmup 1" \
 "300 r5j_bench_synth1m_2048x2048_512spp.json -- python3 bench.py --scene synth1m --width 2048 --height 2048 --spp 512 --steps 1 --warmup 1" \
 "150 r5j_bench_path_caustic_512x512_64spp.json -- python3 bench.py --integrator path --spp 64 --steps 5 --warmup 1" \
 "150 r5j_bench_direct_caustic_512x512_64spp.json -- python3 bench.py --integrator direct --spp 64 --steps 5 --warmup 1" \
 "200 r5j_tail.log -- python3 tools/shard_tail.py caustic 512 512 256 1 8" \
 "250 r5j_bench_rr_hardlight_512x512_1024spp.json -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5e/kt_rr_hl -o kt --output-format csv -- python3 bench.py --russian-roulette --scene hardlight --spp 1024 --steps 2 --warmup 1 --count-spp 16" \
 "420 r5j_bench_rr.json -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5e/kt_rr -o kt --output-format csv -- python3 bench.py --russian-roulette --steps 1 --warmup 0" \
 "300 r5j_bench_rr_second.json -- python3 bench.py --russian-roulette --steps 1 --warmup 0 --no-cpu --no-parity"
