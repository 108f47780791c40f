cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# the final round-5 bench lines (the stamped PMC summaries of gpu_r5final_a.sh are in profiles/)
tools/gpu_steps.sh \
 "200 r5f_bench.json -- python3 bench.py --steps 20 --warmup 2" \
 "200 r5f_bench_hardlight_512x512_1024spp.json -- python3 bench.py --scene hardlight --spp 1024 --steps 5 --warmup 1" \
 "250 r5f_bench_caustic_1024x1024_1024spp.json -- python3 bench.py --width 1024 --height 1024 --spp 1024 --steps 1 --warmup 1" \
 "300 r5f_bench_synth1m_2048x2048_512spp.json -- python3 bench.py --scene synth1m --width 2048 --height 2048 --spp 512 --steps 1 --warmup 1" \
 "150 r5f_bench_path_caustic_512x512_64spp.json -- python3 bench.py --integrator path --spp 64 --steps 5 --warmup 1" \
 "150 r5f_bench_direct_caustic_512x512_64spp.json -- python3 bench.py --integrator direct --spp 64 --steps 5 --warmup 1" \
 "200 r5f_tail.log -- python3 tools/shard_tail.py caustic 512 512 256 1 8" \
 "250 r5f_bench_rr_hardlight_512x512_1024spp.json -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5/kt_rr_hl -o kt --output-format csv -- python3 bench.py --russian-roulette --scene hardlight --spp 1024 --steps 2 --warmup 1 --count-spp 16" \
 "420 r5f_bench_rr.json -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5/kt_rr -o kt --output-format csv -- python3 bench.py --russian-roulette --steps 1 --warmup 0"
