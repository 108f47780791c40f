cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# Russian roulette: three Caustic 512^2x256 frames (walks shared per wave, wave walks in turn), the RR HardLight bench
tools/gpu_steps.sh \
 "200 r5i_rr_c1.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py caustic 512 512 256" \
 "200 r5i_rr_c2.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py caustic 512 512 256" \
 "200 r5i_rr_c3.log -- env RR_PROBE_NO_COUNT=1 python tools/rr_probe.py caustic 512 512 256" \
 "200 r5i_bench_rr_hl.json -- python3 bench.py --russian-roulette --scene hardlight --spp 1024 --steps 2 --warmup 1 --count-spp 16"
