set -e
cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "150 r4b_sweep1.log -- tools/sweep_libs.sh gpurun_out/r4b_sweep.txt default r3 default r3" \
 "60 r4b_nograze.log -- BDPT_GRAZE_CODES=0 python bench.py --no-cpu --no-parity --steps 3 --warmup 1" \
 "60 r4b_default2.log -- python bench.py --no-cpu --no-parity --steps 3 --warmup 1" \
 "60 r4b_nograze2.log -- BDPT_GRAZE_CODES=0 python bench.py --no-cpu --no-parity --steps 3 --warmup 1" \
 "100 r4b_rr_small.log -- python tools/rr_probe.py caustic 512 512 1" \
 "150 r4b_rr_l4.log -- python tools/rr_probe.py caustic 512 512 256 45 64"
