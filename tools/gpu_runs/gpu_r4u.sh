cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "300 r4u_tail.log -- bash tools/tail_sweep.sh gpurun_out/r4u_tail.txt default rev tc8 default rev tc8 -- caustic 512 512 256 1 8" \
 "300 r4u_synth.log -- python3 bench.py --no-cpu --no-parity --scene synth1m --steps 2 --warmup 1" \
 "400 r4u_rr_hl.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py hardlight 512 512 64"
