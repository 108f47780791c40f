cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "200 r4aa_bench.json -- python3 bench.py --steps 20 --warmup 2" \
 "200 r4aa_bench_hardlight_512x512_1024spp.json -- python3 bench.py --scene hardlight --spp 1024 --steps 5 --warmup 1" \
 "200 r4aa_bench_caustic_1024x1024_1024spp.json -- python3 bench.py --width 1024 --height 1024 --spp 1024 --steps 1 --warmup 1" \
 "300 r4aa_bench_synth1m_2048x2048_512spp.json -- python3 bench.py --scene synth1m --width 2048 --height 2048 --spp 512 --steps 1 --warmup 1" \
 "200 r4aa_bench_path_caustic_512x512_64spp.json -- python3 bench.py --integrator path --spp 64 --steps 5 --warmup 1" \
 "200 r4aa_bench_direct_caustic_512x512_64spp.json -- python3 bench.py --integrator direct --spp 64 --steps 5 --warmup 1"
