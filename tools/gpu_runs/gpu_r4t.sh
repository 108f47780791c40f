cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r4t
tools/gpu_steps.sh \
 "300 r4t_bench_rr_hl.log -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4t/kt_rr_hl -o kt --output-format csv -- python3 bench.py --russian-roulette --scene hardlight --spp 1024 --steps 2 --warmup 1" \
 "800 r4t_bench_rr.log -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4t/kt_rr -o kt --output-format csv -- python3 bench.py --russian-roulette --steps 1 --warmup 0"
