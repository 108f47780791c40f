cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_fb
# Russian-roulette bench lines (rocprofv3 kernel trace of each), the synth1m profile and bench line
tools/gpu_steps.sh \
 "300 fb_bench_rr.json -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fb/kt_rr -o kt --output-format csv -- python3 bench.py --russian-roulette --steps 1 --warmup 0" \
 "200 fb_bench_rr_hardlight_512x512_1024spp.json -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fb/kt_rr_hl -o kt --output-format csv -- python3 bench.py --russian-roulette --scene hardlight --spp 1024 --steps 2 --warmup 1" \
 "400 fb_prof_synth.log -- bash tools/profile_round.sh fb synth1m 2048 2048 512" \
 "20 fb_copy.log -- cp gpurun_out/prof_fb/pmc_*.json profiles/" \
 "250 fb_bench_synth1m_2048x2048_512spp.json -- python3 bench.py --scene synth1m --width 2048 --height 2048 --spp 512 --steps 1 --warmup 1"
