cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# GPU suite on the fma-slab default; the translated-scene cases on the slab_fast build too
tools/gpu_steps.sh \
 "400 r5q_gpu_tests.log -- python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "150 r5q_translated_nofma.log -- BDPT_AMD_LIB=$GRAFT_REPO_ROOT/bidirectional-path-tracing_amd/lib/libbdpt_amd_nofma.so python -u -m pytest tests/test_gpu_parity.py -k 'translated or far_camera' -q --timeout 120 --timeout-method thread"
