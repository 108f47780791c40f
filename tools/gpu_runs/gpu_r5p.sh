cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# the fma slab as the default (BDPT_SLAB_FMA 2): GPU suite, the translated-scene test on the
# slab_fast build too (nofma), parity-checked bench lines
tools/gpu_steps.sh \
 "400 r5p_gpu_tests.log -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "150 r5p_translated_nofma.log -- BDPT_AMD_LIB=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib/libbdpt_amd_nofma.so python -u -m pytest tests/test_gpu_parity.py -k 'translated or far_camera' -x -q --timeout 120 --timeout-method thread" \
 "200 r5p_bench.json -- python3 bench.py --steps 10 --warmup 2" \
 "200 r5p_bench_hardlight.json -- python3 bench.py --scene hardlight --spp 1024 --steps 5 --warmup 1"
