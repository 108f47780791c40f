cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "120 r4i_sweep.log -- tools/sweep_libs.sh gpurun_out/r4i_sweep.txt default gd va r3 default gd va r3" \
 "500 r4i_bench_rr.log -- python bench.py --russian-roulette --steps 1 --warmup 0"
