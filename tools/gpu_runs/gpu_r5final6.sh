cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# synth1m (configs[4]) on the deep-scene threshold 36: its stamped profile (copied into profiles/ on the
# box) and its bench line; the host change does not touch the kernel build
tools/gpu_steps.sh \
 "500 r5k_prof_synth.log -- bash tools/profile_round.sh r5f synth1m 2048 2048 512" \
 "30 r5k_copy.log -- cp gpurun_out/prof_r5f/pmc_*synth1m*.json profiles/ && ls -la profiles/pmc_*synth1m*" \
 "300 r5k_bench_synth1m_2048x2048_512spp.json -- python3 bench.py --scene synth1m --width 2048 --height 2048 --spp 512 --steps 1 --warmup 1" \
 "200 r5k_gpu_tests_large.log -- python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -k synth -x -q --timeout 150 --timeout-method thread"
