cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r4m
tools/gpu_steps.sh \
 "1000 r4m_bench_rr.log -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4m/kt_rr -o kt --output-format csv -- python3 bench.py --russian-roulette --steps 1 --warmup 0"
