cd $GRAFT_REPO_ROOT
# final build: GPU suite, smoke, caustic + hardlight profiles, then the bench lines
# (the profiles copied into profiles/ on the box so bench.py stamps traffic / issue)
tools/gpu_steps.sh \
 "300 fa_gpu_tests.log -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "120 fa_smoke.log -- python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "300 fa_prof_caustic.log -- bash tools/profile_round.sh fa caustic 512 512 256" \
 "300 fa_prof_hl.log -- bash tools/profile_round.sh fa hardlight 512 512 1024" \
 "20 fa_copy.log -- cp gpurun_out/prof_fa/pmc_*.json profiles/" \
 "200 fa_bench.json -- python3 bench.py --steps 20 --warmup 2" \
 "200 fa_bench_hardlight_512x512_1024spp.json -- python3 bench.py --scene hardlight --spp 1024 --steps 5 --warmup 1" \
 "200 fa_bench_caustic_1024x1024_1024spp.json -- python3 bench.py --width 1024 --height 1024 --spp 1024 --steps 1 --warmup 1" \
 "150 fa_bench_path_caustic_512x512_64spp.json -- python3 bench.py --integrator path --spp 64 --steps 5 --warmup 1" \
 "150 fa_bench_direct_caustic_512x512_64spp.json -- python3 bench.py --integrator direct --spp 64 --steps 5 --warmup 1"
